// nr_fwd.h -- forward: k_face_setup, k_vertex_normals, k_raster_fwd (face-index map), standalone k_tex_pack
// Part of nr_raster.hip (one translation unit); see that file and DESIGN.md.
#pragma once

#pragma clang fp contract(off)

namespace {

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
                                                    int uv_items, float* __restrict__ fnorm, TexPack pk, ZeroFill zf,
                                                    uint8_t* __restrict__ bin_part, int xcd_items, int sparse_groups) {
    __shared__ int2 s_bb[SETUP_FACES];
    // the block's face records, assembled per face and then written out coalesced (a record per lane
    // would store 64-B strided rows); the bin-mask words reuse the space afterwards
    extern __shared__ __attribute__((aligned(16))) float s_stage[];  // setup_lds_words(nbins) floats
    float* s_frec = s_stage;
    uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_stage);
    // xcd_items (B % 8 == 0): block L works on item (L & 7) + 8 (j / groups), face group j % groups
    // (j = L >> 3): workgroups are dealt to XCD L % 8, so all of an item's blocks write through one L2,
    // where the 24-B pieces that neighbouring face groups write into each bin's mask row meet in whole
    // lines before they go to HBM (spread over eight L2s, each piece went out as a partial line)
    int b, grp;
    if (xcd_items) {
        const int L = blockIdx.y * gridDim.x + blockIdx.x, j = L >> 3;
        b = (L & 7) + 8 * (j / gridDim.x);
        grp = j % gridDim.x;
    } else {
        // (round 6: the (item, group) tasks in 8 contiguous chunks, one per XCD, so that neighbouring
        // face groups' mask pieces would meet in one L2 for other batch sizes too: the torus and teapot
        // setups measured the same, 16.2-16.4 / 10.6-10.7 us, gpurun_out/chunk; not kept)
        b = blockIdx.y;
        grp = blockIdx.x;
    }
    const int f0 = grp * SETUP_FACES;
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
                bool fxyz = true, fzq = true, zeq = true;
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    fxyz = fxyz && coord_ok(c[3 * k]) && coord_ok(c[3 * k + 1]) && in_range(c[3 * k + 2], 0x1p-20f, 0x1p20f);
                    fzq = fzq && in_range(c[3 * k + 2] + 1e-10f, 0x1p-20f, 0x1p20f);
                    zeq = zeq && (c[3 * k + 2] + 1e-10f == c[3 * k + 2]);
                }
                const int flags = (fxyz ? FACE_FAST_XYZ : 0) | (fzq ? FACE_FAST_ZQ : 0) | (zeq ? FACE_ZQ_EQ : 0);
                float4* rec = reinterpret_cast<float4*>(s_frec + t * FACE_REC);
                rec[0] = make_float4(c[0], c[1], c[2], c[3]);
                rec[1] = make_float4(c[4], c[5], c[6], c[7]);
#ifdef NR_REC48
                rec[2] = make_float4(c[8], __int_as_float(flags), 0.f, 0.f);
#else
                rec[2] = make_float4(c[8], face_rcp(c[2]), face_rcp(c[5]), face_rcp(c[8]));
                rec[3] = make_float4(face_rcp(c[2] + 1e-10f), face_rcp(c[5] + 1e-10f), face_rcp(c[8] + 1e-10f),
                                     __int_as_float(flags));
#endif
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
            (void)bbox;  // the pixel bbox stays in LDS (the masks); the forward stages float bounds itself
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
    const int w0 = grp * (SETUP_FACES / 32);
    const int nw = min(SETUP_FACES / 32, nwords - w0);
    if (nbins * (SETUP_FACES / 32) <= SETUP_LDS_WORDS) {  // (setup_lds_words sized s_stage for this)
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
        if (sparse_groups && bin_part) {
            // (k_bin_order's group lists) a thread per bin writes the group's count and, only where it
            // has candidates, its words: the forward reads no other piece
            uint8_t* row = bin_part + ((long long)b * gridDim.x + grp) * nbins;
            for (int bin = t; bin < nbins; bin += blockDim.x) {
                const uint32_t* sm = s_mask + bin * (SETUP_FACES / 32);
                int pc = 0;
#pragma unroll
                for (int wi = 0; wi < SETUP_FACES / 32; wi++) pc += __builtin_popcount(sm[wi]);
                row[bin] = (uint8_t)pc;
                if (pc)
                    for (int wi = 0; wi < nw; wi++) mask[((long long)b * nbins + bin) * nwords + w0 + wi] = sm[wi];
            }
            zero_fill(zf);
            return;
        }
        for (int p = t; p < nbins * nw; p += blockDim.x) {
            const int bin = p / nw, wi = p % nw;
            mask[((long long)b * nbins + bin) * nwords + w0 + wi] = s_mask[bin * (SETUP_FACES / 32) + wi];
        }
        if (bin_part) {
            // this face group's candidate faces per bin (at most SETUP_FACES: a byte), a row of
            // [B, groups, nbins] that k_bin_order sums over the groups for the deep-first order: every
            // entry is written, so the counts need no zero fill (a memset launch per forward until v56)
            // and no atomics
            uint8_t* row = bin_part + ((long long)b * gridDim.x + grp) * nbins;
            for (int bin = t; bin < nbins; bin += blockDim.x) {
                int pc = 0;
#pragma unroll
                for (int wi = 0; wi < SETUP_FACES / 32; wi++) pc += __builtin_popcount(s_mask[bin * (SETUP_FACES / 32) + wi]);
                row[bin] = (uint8_t)pc;
            }
        }
        zero_fill(zf);
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
    zero_fill(zf);
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
// Deep-first dispatch order of the forward's bins (deep-bin launches: the car, the 50k torus).  A bin
// with thousands of candidate faces keeps its block for 100-500 us while a shallow bin's lasts a few;
// dispatched in screen order, the deepest bins of the car started up to 360 us into a 790 us kernel and
// the kernel ended on them (profiles/r04_*_fwd_wave_phases_car.txt).  This orders the (item, bin)
// pairs by candidate count, descending, in log2 buckets (a stable counting sort: screen order within a
// bucket), longest first: one list per XCD when B is a multiple of 8 (list x: items = x mod 8, read by
// the blocks dealt to XCD x, ordered_bin), else one list.  Any order gives the same results: every
// bin's block is independent.
// buckets of the candidate count, deepest = highest: one per octave (0 for none)
constexpr int ORDER_BUCKETS = 16;
__device__ __forceinline__ int count_bucket(int c) { return c <= 0 ? 0 : min(ORDER_BUCKETS - 1, 32 - __clz(c)); }
// one block of 1024 threads per list, a stable counting sort: each wave takes 64-entry chunks and counts
// its chunk's buckets with ballots; the per-(chunk, bucket) counts become output offsets (deepest
// bucket first, chunks in list order); each entry then goes to its chunk's offset plus its rank among
// the chunk's lanes of the same bucket.  Stable: screen order (and so neighbouring bins, which share
// face records in L2) within a bucket -- an unstable order cost the car's forward ~6 us.
constexpr int ORDER_MAX_ENTRIES = 64 * 256;
constexpr int ORDER_SLICED_MAX = 2048;  // k_bin_order: lists of up to 2 x 1024 entries are summed in slices
// (ORDER_EMPTY, the entry flag of a bin without candidates, is in nr_common.h with ordered_bin)
// split (optional): per list, the length of its prefix of bins with >= 2^(split_bucket - 1) candidate
// faces, at most cap (the deep launch of a split forward, run_face_index)
// parts: the setup's per-(item, face group, bin) candidate counts [B, groups, nbins] (k_face_setup)
__global__ __launch_bounds__(1024) void k_bin_order(const uint8_t* __restrict__ parts, int groups, int* __restrict__ order,
                                                    int B, int nbins, int* __restrict__ split, int split_bucket, int cap) {
    __shared__ int s_h[ORDER_MAX_ENTRIES / 64][ORDER_BUCKETS];
    __shared__ int s_base[ORDER_BUCKETS];
    __shared__ uint8_t s_bk[ORDER_MAX_ENTRIES];  // each entry's count bucket
    const bool per_xcd = gridDim.x == 8;
    const int x = blockIdx.x;
    const int items = per_xcd ? B / 8 : B;
    const int n = items * nbins;
    const int nch = (n + 63) / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int* __restrict__ out = order + (per_xcd ? x * n : 0);
    auto entry = [&](int k) {
        const int j = k / nbins;
        return (per_xcd ? x + 8 * j : j) * nbins + (k - j * nbins);
    };
    // each entry's candidate count, the face groups' counts summed, as its bucket: four consecutive
    // bins of an item per thread and 32-bit loads when the bins come in fours (a multiple of 4 per item)
    // (fewer quads than threads, e.g. one item's bins: S threads per quad share its groups, the loads of
    // a quad's S slices in flight at once, summed in LDS -- the torus's one list of 256 quads over 261
    // groups took 20.6 us a thread per quad)
    const int quads = nbins % 4 == 0 ? n / 4 : 0;
    int S = 1;
    while (quads > 0 && S < 8 && 2 * S * quads <= (int)blockDim.x) S *= 2;
    if (S > 1) {
        __shared__ int s_cnt[ORDER_SLICED_MAX];
        for (int k = threadIdx.x; k < n; k += blockDim.x) s_cnt[k] = 0;
        __syncthreads();
        const int q = threadIdx.x % quads, sl = threadIdx.x / quads;
        if (sl < S) {
            const int k = 4 * q, e = entry(k), b = e / nbins, bin = e - b * nbins;
            const uint32_t* p = reinterpret_cast<const uint32_t*>(parts + (long long)b * groups * nbins + bin);
            int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll 8
            for (int gr = sl; gr < groups; gr += S) {
                const uint32_t v = p[(long long)gr * (nbins / 4)];
                c0 += v & 0xffu;
                c1 += (v >> 8) & 0xffu;
                c2 += (v >> 16) & 0xffu;
                c3 += v >> 24;
            }
            atomicAdd(&s_cnt[k], c0);
            atomicAdd(&s_cnt[k + 1], c1);
            atomicAdd(&s_cnt[k + 2], c2);
            atomicAdd(&s_cnt[k + 3], c3);
        }
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += blockDim.x) s_bk[k] = (uint8_t)count_bucket(s_cnt[k]);
    } else if (nbins % 4 == 0) {
        for (int q = threadIdx.x; q < n / 4; q += blockDim.x) {
            const int k = 4 * q, e = entry(k), b = e / nbins, bin = e - b * nbins;
            const uint32_t* p = reinterpret_cast<const uint32_t*>(parts + (long long)b * groups * nbins + bin);
            int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll 8
            for (int gr = 0; gr < groups; gr++) {
                const uint32_t v = p[(long long)gr * (nbins / 4)];
                c0 += v & 0xffu;
                c1 += (v >> 8) & 0xffu;
                c2 += (v >> 16) & 0xffu;
                c3 += v >> 24;
            }
            s_bk[k] = (uint8_t)count_bucket(c0);
            s_bk[k + 1] = (uint8_t)count_bucket(c1);
            s_bk[k + 2] = (uint8_t)count_bucket(c2);
            s_bk[k + 3] = (uint8_t)count_bucket(c3);
        }
    } else {
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            const int e = entry(k), b = e / nbins, bin = e - b * nbins;
            const uint8_t* p = parts + (long long)b * groups * nbins + bin;
            int c = 0;
#pragma unroll 8
            for (int gr = 0; gr < groups; gr++) c += p[(long long)gr * nbins];
            s_bk[k] = (uint8_t)count_bucket(c);
        }
    }
    __syncthreads();
    for (int ch = wid; ch < nch; ch += nw) {
        const int k = ch * 64 + lane;
        const int bk = k < n ? (int)s_bk[k] : -1;
#pragma unroll
        for (int b = 0; b < ORDER_BUCKETS; b++) {
            const int c = __popcll(__ballot(bk == b));
            if (lane == 0) s_h[ch][b] = c;
        }
    }
    __syncthreads();
    if (threadIdx.x < ORDER_BUCKETS) {  // bucket totals
        int tot = 0;
        for (int ch = 0; ch < nch; ch++) tot += s_h[ch][threadIdx.x];
        s_base[threadIdx.x] = tot;
    }
    __syncthreads();
    if (threadIdx.x < ORDER_BUCKETS) {  // this bucket's chunk offsets: buckets deepest first
        const int b = threadIdx.x;
        int base = 0;
        for (int bb = ORDER_BUCKETS - 1; bb > b; bb--) base += s_base[bb];
        for (int ch = 0; ch < nch; ch++) {
            const int c = s_h[ch][b];
            s_h[ch][b] = base;
            base += c;
        }
    }
    __syncthreads();
    for (int ch = wid; ch < nch; ch += nw) {
        const int k = ch * 64 + lane;
        const int e = k < n ? entry(k) : 0;
        const int bk = k < n ? (int)s_bk[k] : -1;
        int rank = 0;
#pragma unroll
        for (int b = 0; b < ORDER_BUCKETS; b++) {
            const unsigned long long m = __ballot(bk == b);
            if (bk == b) rank = __popcll(m & lt);
        }
        if (k < n) out[s_h[ch][bk] + rank] = e | (bk == 0 ? ORDER_EMPTY : 0);
    }
    if (split && threadIdx.x == 0) {  // (s_base still holds the bucket totals)
        int d = 0;
        for (int bb = split_bucket; bb < ORDER_BUCKETS; bb++) d += s_base[bb];
        split[x] = min(d, cap);
    }
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
//      across rounds; the test is split into a per-face pass test and a deferred commit
//      (face_commit), and the deep-bin variant first drops faces whose edge tests fail over the
//      whole 8x8 block (block_culled);
//   4. SHADE: the block then shades its bin's 16x16 output pixels (k_shade's work, shade_quad) from
//      the winners it has just found; otherwise k_shade does it in a launch of its own.
//   Block sizes (picked per launch, run_face_index): 256 threads = 4 waves, each walking the four 8x8
//   blocks of a 16x16 quadrant (most per-thread work, least fixed cost per pixel: best when the grid
//   has many bins of moderate depth, e.g. the headline); 1024 threads = 16 waves, one 8x8 block each
//   (the bin's walks run 4x wider: small batches, where the grid is a few blocks per CU, and dense
//   bins -- 300+ faces over one 8x8 block on a 50k-face torus -- no longer serialise on 4 waves).
//   LDS face record, structure of arrays (float4 i of staged face j at s_face[i * FCAP + j]: the
//   staging stores are lane-contiguous), 7 x float4; the pass test reads rows 0-4 (the depth and bbox
//   tests rows 0-1, issued first), the commit rows 1 and 3-6:
//     0: xmin xmax ymin ymax | 1: zmin k0 k2 k1 | 2: y0 y2 x0 x2 | 3: A=x1-x0 E=x0-x2 B=y1-y0 F=y0-y2
//     4: y1 x1 C=x2-x1 D=y2-y1 | 5: z0 z1 z2 id | 6: 1/z0 1/z1 1/z2 ok
//   (y1-y2 = -D etc. exactly, so w0 = (yp*C - xp*D) + k0 reproduces .cu:130 bit for bit).  The edge
//   tests and weights are scalar f32 instructions: packed ones (v_pk_*_f32, v42-v45) issue in 4
//   cycles, the rate of two scalar ones, and their operand pairs cost copies of xp and yp (scalar:
//   headline fwd 0.157 -> 0.152 ms, same-box A/B).
constexpr int FREC = 7;  // float4 per staged face
// staged faces per round: 160 for the 256-thread variant (8 blocks per CU need <= 20 KB of LDS;
// 128 -> 160: headline fwd 0.208 -> 0.195 ms), 512 for the 1024-thread one (2 blocks per CU: up to
// 80 KB each; 256 -> 512: car fwd 0.914 -> 0.81 ms, torus 0.151 -> 0.132 ms)
template <int NTF> struct FwdCfg {
    static_assert(NTF == 256 || NTF == 1024, "forward block sizes");
    static constexpr int NW = NTF / 64;                        // waves
    static constexpr int NSUB = (COARSE * COARSE) / NTF;       // 8x8 blocks (pixels) per thread
    static constexpr int CAND = NTF >= 1024 ? 1024 : 512;      // candidate ids expanded per round
    static constexpr int FCAP = NTF >= 1024 ? 512 : 160;       // faces staged per round
    // staged records, candidate ids (dyn + SHADE: then the winners' staging slots), block masks, block
    // extents; (1024 threads) the dealt-quarter walk's quarter masks, quarter extents, per-pixel state
    // and per-quarter counts / order
    static constexpr int LDS_BASE = FCAP * FREC * 16 + CAND * 4 + FCAP * 2 + 16 * 4;
    static constexpr int LDS_DQ = NTF >= 1024 ? FCAP * 8 + 32 * 4 + COARSE * COARSE * 8 + 64 * 4 * 2 : 0;
    static constexpr int LDS = LDS_BASE + LDS_DQ;
    // 8x8 block k of wave w: its origin (ox, oy) in the bin
    __device__ static __forceinline__ void block_of(int w, int k, int& ox, int& oy) {
        if (NSUB == 1) {         // 16 waves: wave w owns block (w & 3, w >> 2)
            ox = (w & 3) * 8;
            oy = (w >> 2) * 8;
        } else {                 // 4 waves: the 16x16 quadrant w, walked as four 8x8 blocks
            ox = (w & 1) * 16 + (k & 1) * 8;
            oy = (w >> 1) * 16 + (k >> 1) * 8;
        }
    }
};

// The staged record rows of one walked face: the pass test's rows 0-4 are loaded together, before the
// first test (one LDS round trip; with the loads sunk into the test stages each stage waited for its
// own: 2 -> 6 eager rows of the earlier 8-row layout took the headline forward 0.268 -> 0.259 ms, the
// car 1.20 -> 1.14 ms).  FST = the SoA stride (FCAP).
constexpr int FWD_EAGER = 5;
template <int FST>
struct FaceRows {
    float4 r[FREC];
    __device__ __forceinline__ void load(const float4* e) {
#pragma unroll
        for (int i = 0; i < FWD_EAGER; i++) r[i] = e[i * FST];
        // an empty asm that takes the rows keeps the compiler from sinking each load into the branch
        // that first uses it (which costs an LDS round trip per test stage)
#pragma unroll
        for (int i = 0; i < FWD_EAGER; i++) asm volatile("" ::"v"(r[i].x), "v"(r[i].y), "v"(r[i].z), "v"(r[i].w));
    }
    __device__ __forceinline__ float4 get(const float4* e, int i) const { return i < FWD_EAGER ? r[i] : e[i * FST]; }
};
// The reference's per-face test sequence (.cu:94-148) in deferred form: the walk runs only the
// state-independent part of the test per face (the pass test: .cu:94-116, with the depth reject of
// .cu:124-126 against a bound >= the pixel's current minimum, so a face it rejects the exact test
// rejects too), and keeps per pixel the one face that passed it and is not yet committed; the rest of
// the test -- depth reject, barycentric division chain, near / far and the z-test (face_commit) -- runs
// for all pending pixels of the wave at once, when a newly walked face passes at a pixel that already
// has a pending face, and at the end of the block's walk. Every pixel still commits its faces in
// ascending order with the state the sequential loop has at that point (what was pending has been
// committed before), so the result is that of .cu:82-149; the division chain, run by the whole wave
// for any one passing lane, runs about a third as often on the headline.
// .cu:124-148 for a face that passed the pass test at this pixel (slot: its staging slot, per lane);
// the winner is recorded as its face id, or (SLOT) as its staging slot
template <int FST, bool SLOT>
__device__ __forceinline__ void face_commit(const float4* s_face, int slot, float xp, float yp, float near, float far,
                                            float delta, float& depth_min, int& best) {
    const float4* e = s_face + slot;
    const float4 q1 = e[1 * FST];
    // every row in one LDS round trip (the depth reject would otherwise wait for row 1 first)
    const float4 q3 = e[3 * FST], q4 = e[4 * FST], q5 = e[5 * FST], q6 = e[6 * FST];
    asm volatile("" ::"v"(q3.x), "v"(q3.y), "v"(q3.z), "v"(q3.w), "v"(q4.z), "v"(q4.w), "v"(q1.y), "v"(q1.z));
    asm volatile("" ::"v"(q1.w), "v"(q5.x), "v"(q5.y), "v"(q5.z), "v"(q5.w), "v"(q6.x), "v"(q6.y), "v"(q6.z), "v"(q6.w));
    if (depth_min < q1.x) return;
    const float z0 = q5.x, z1 = q5.y, z2 = q5.z;
    // .cu:130-132: w2 = (yp A - xp B) + k2, w1 = (yp E - xp F) + k1, w0 = (yp C - xp D) + k0
    float w2 = (yp * q3.x - xp * q3.z) + q1.z;
    float w1 = (yp * q3.y - xp * q3.w) + q1.w;
    float w0 = (yp * q4.z - xp * q4.w) + q1.y;
    const float ws = w0 + w1 + w2;
    float zp;
    if (__float_as_int(q6.w) && in_range(ws, 0x1p-20f, 0x1p20f)) {  // as face_test
        const float rs = rcp_nr(ws);
        w0 = div_nr(w0, ws, rs);
        w1 = div_nr(w1, ws, rs);
        w2 = div_nr(w2, ws, rs);
        const float sum = div_nr(w0, z0, q6.x) + div_nr(w1, z1, q6.y) + div_nr(w2, z2, q6.z);
        if (in_range(sum, 0x1p-90f, 0x1p90f)) {
            const float r = rcp_nr(sum);
            zp = __builtin_fmaf(__builtin_fmaf(-sum, r, 1.f), r, r);
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
    if (zp <= depth_min - delta) {
        depth_min = zp;
        best = SLOT ? slot : __float_as_int(q5.w);
    }
}

constexpr int ZCULL_MIN = 512;  // candidates of a bin (first bin-mask round)
#ifndef NR_ZREFRESH
#define NR_ZREFRESH 255
#endif
// one wave's walk of the n staged faces over its 8x8 block u of the bin (pixel (xp, yp) per lane): the
// ballot takes the staged faces whose block mask (face_block_mask: bbox, and with CULL the edge cull)
// has bit u, then the per-face test runs in ascending order
#ifdef NR_COUNT_TESTS
// diagnostic build: face tests, faces walked, commit batches, walks (nr_count_read)
__device__ unsigned long long g_fwd_count[4];
#endif
template <int FST, bool SLOT, bool ZCULL = false, typename MT = uint16_t, bool Q16 = false>
__device__ __forceinline__ void walk_block(const float4* __restrict__ s_face, const MT* __restrict__ s_bm, int u,
                                           int n, int lane, float xp, float yp, float near, float far, float delta,
                                           float& depth_min, int& best) {
    int pend = -1;               // staging slot of my pixel's pending face
    unsigned long long occ = 0;  // the wave's pixels with a pending face
    // (ZCULL: the deep variant's bins of >= ZCULL_MIN candidates) a face whose nearest corner lies
    // behind every pixel's current depth (the wave's maximum, refreshed when a commit has changed a
    // depth since, at most every NR_ZREFRESH + 1 faces) fails the pass test's depth reject at each of
    // them (depth_min only decreases; NaN bounds are kept): it is dropped in the ballot, with 63
    // others, instead of walked alone.  Car forward 0.625 -> 0.601 ms; the 50k torus (deep bins of low
    // depth complexity) 0.118 -> 0.120 ms; on every bin of the headline and the torus the gate-free
    // version cost +4 us each (same-box A/Bs, gpurun_out/o4-o9).
    float zmax = 0.f;
    bool dirty = true;  // (wave-uniform) a commit may have lowered a depth since zmax was taken
#ifdef NR_COUNT_TESTS
    unsigned long long cnt_walked = 0, cnt_commits = 0;
#endif
    for (int c0 = 0; c0 < n; c0 += 64) {
        if (ZCULL && dirty && (c0 & NR_ZREFRESH) == 0) {
            zmax = wave_max(depth_min);
            dirty = false;
        }
        bool hit = false;
        if (c0 + lane < n) {
            hit = (s_bm[c0 + lane] >> u) & 1;
            if (ZCULL) hit = hit && !(s_face[FST + c0 + lane].x > zmax);
        }
        // faces touching this wave's pixels, walked in ascending order
        for (unsigned long long m = __ballot(hit); m; m &= m - 1) {
            const int slot = c0 + __builtin_ctzll(m);
            const float4* e = s_face + slot;
#ifdef NR_COUNT_TESTS
            cnt_walked++;
#endif
            FaceRows<FST> fr;
            fr.load(e);
            // the pass test with its outcome kept as a wave mask: the depth and bbox tests of every lane
            // form one mask, the edge tests run only when a lane is left (a uniform branch), and the
            // pending slot is set from the mask directly (no per-lane boolean to rebuild a ballot from)
            const float4 q0 = fr.get(e, 0), q1 = fr.get(e, 1);
            // each comparison straight to a lane mask (v_cmp into an SGPR pair; the masks combine on the
            // scalar unit): a ballot of the combined boolean costs a v_cndmask + v_cmp per face to
            // rebuild the mask.  !(a < b) is "a >= b or unordered" (UGE), !(a > b) is ULE.
            // (Q16: a 4x4 quarter, lanes 0-15 only)
            const unsigned long long pre = lane_mask_uge(depth_min, q1.x) & lane_mask_uge(xp, q0.x) &
                                           lane_mask_ule(xp, q0.y) & lane_mask_uge(yp, q0.z) & lane_mask_ule(yp, q0.w) &
                                           (Q16 ? 0xffffull : ~0ull);
            unsigned long long cov = 0;
            if (pre) {
                // .cu:107-116: c1 = (yp - y0) A - B (xp - x0), c3 = (yp - y2) E - F (xp - x2),
                // c2 = (yp - y1) C - (xp - x1) D; pass unless c1 c2 < 0 or c2 c3 < 0
                const float4 q2 = fr.get(e, 2), q3 = fr.get(e, 3), q4 = fr.get(e, 4);
                const float c1 = (yp - q2.x) * q3.x - q3.z * (xp - q2.z);
                const float c3 = (yp - q2.y) * q3.y - q3.w * (xp - q2.w);
                const float c2 = (yp - q4.x) * q4.z - (xp - q4.y) * q4.w;
                cov = lane_mask_uge(c1 * c2, 0.f) & lane_mask_uge(c3 * c2, 0.f) & pre;
            }
            if (cov & occ) {  // commit first where this face would queue behind a pending one
#ifdef NR_COUNT_TESTS
                cnt_commits++;
#endif
                if (pend >= 0) face_commit<FST, SLOT>(s_face, pend, xp, yp, near, far, delta, depth_min, best);
                pend = -1;
                occ = 0;
                dirty = true;
            }
            {
                int sv = slot;
                asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(pend) : "v"(pend), "v"(sv), "s"(cov));
            }
            occ |= cov;
        }
    }
#ifdef NR_COUNT_TESTS
    if (occ) cnt_commits++;
    if (lane == 0) {
        atomicAdd(&g_fwd_count[0], cnt_walked * (Q16 ? 16ull : 64ull));
        atomicAdd(&g_fwd_count[1], cnt_walked);
        atomicAdd(&g_fwd_count[2], cnt_commits);
        atomicAdd(&g_fwd_count[3], 1ull);
    }
#endif
    if (pend >= 0) face_commit<FST, SLOT>(s_face, pend, xp, yp, near, far, delta, depth_min, best);
}

// walk_block for one 4x4 quarter q (the dealt-quarter deep walk) with four faces per step: lane group
// g = lane >> 4 runs the pass test of the step's g-th face (ballot order, so ascending) at pixel
// lane & 15, every group holding the same 16 pixels (xp, yp, depth_min replicated by the caller).  The
// groups' coverage masks then go through the pending-face logic one group at a time, in face order, on
// the scalar unit: a face that passes at a pixel with a pending face commits the wave's pending faces
// first, exactly as walk_block's sequential loop does, so every pixel still commits its faces in
// ascending order (face_commit: lanes 0-15, whose depth_min and best are the pixels' own).  Groups 1-3
// test against a copy of the depths taken before the step's commits -- a bound >= the pixel's current
// minimum, as the pass test allows -- refreshed from lanes 0-15 after any commit.  With one face per
// step lanes 16-63 sat idle through the quarter walk; this walks the deep bins' quarters in about a
// quarter of the steps.
template <int FST>
__device__ __forceinline__ void walk_quarter4(const float4* __restrict__ s_face, const uint64_t* __restrict__ s_q, int q,
                                              int n, int lane, float xp, float yp, float near, float far, float delta,
                                              float& depth_min, int& best) {
    int pend = -1;               // staging slot of my pixel's pending face (lanes 0-15)
    unsigned long long occ = 0;  // the quarter's pixels (bits 0-15) with a pending face
    float zmax = 0.f;
    bool dirty = true;
    const int g = lane >> 4;
#ifdef NR_COUNT_TESTS
    unsigned long long cnt_walked = 0, cnt_commits = 0;
#endif
    for (int c0 = 0; c0 < n; c0 += 64) {
        if (dirty && (c0 & NR_ZREFRESH) == 0) {  // (as walk_block's ZCULL)
            zmax = wave_max(depth_min);
            dirty = false;
        }
        bool hit = false;
        if (c0 + lane < n) hit = ((s_q[c0 + lane] >> q) & 1) && !(s_face[FST + c0 + lane].x > zmax);
        for (unsigned long long m = __ballot(hit); m;) {
            int sl[4];
            unsigned long long valid = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                sl[k] = m ? c0 + __builtin_ctzll(m) : c0;
                valid |= m ? 0xffffull << (16 * k) : 0ull;
                m &= m - 1;
            }
#ifdef NR_COUNT_TESTS
            cnt_walked += __popcll(valid) >> 4;
#endif
            const int slot = g == 0 ? sl[0] : g == 1 ? sl[1] : g == 2 ? sl[2] : sl[3];
            const float4* e = s_face + slot;
            FaceRows<FST> fr;
            fr.load(e);
            const float4 q0 = fr.get(e, 0), q1 = fr.get(e, 1);
            const unsigned long long pre = lane_mask_uge(depth_min, q1.x) & lane_mask_uge(xp, q0.x) &
                                           lane_mask_ule(xp, q0.y) & lane_mask_uge(yp, q0.z) & lane_mask_ule(yp, q0.w) &
                                           valid;
            unsigned long long cov = 0;
            if (pre) {
                const float4 q2 = fr.get(e, 2), q3 = fr.get(e, 3), q4 = fr.get(e, 4);
                const float c1 = (yp - q2.x) * q3.x - q3.z * (xp - q2.z);
                const float c3 = (yp - q2.y) * q3.y - q3.w * (xp - q2.w);
                const float c2 = (yp - q4.x) * q4.z - (xp - q4.y) * q4.w;
                cov = lane_mask_uge(c1 * c2, 0.f) & lane_mask_uge(c3 * c2, 0.f) & pre;
            }
            if (cov) {
                bool committed = false;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const unsigned long long ck = (cov >> (16 * k)) & 0xffffull;
                    if (ck & occ) {
#ifdef NR_COUNT_TESTS
                        cnt_commits++;
#endif
                        if (pend >= 0) face_commit<FST, false>(s_face, pend, xp, yp, near, far, delta, depth_min, best);
                        pend = -1;
                        occ = 0;
                        committed = true;
                    }
                    int sv = sl[k];
                    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(pend) : "v"(pend), "v"(sv), "s"(ck));
                    occ |= ck;
                }
                if (committed) {
                    depth_min = __shfl(depth_min, lane & 15);
                    dirty = true;
                }
            }
        }
    }
#ifdef NR_COUNT_TESTS
    if (occ) cnt_commits++;
    if (lane == 0) {
        atomicAdd(&g_fwd_count[0], cnt_walked * 16ull);
        atomicAdd(&g_fwd_count[1], cnt_walked);
        atomicAdd(&g_fwd_count[2], cnt_commits);
        atomicAdd(&g_fwd_count[3], 1ull);
    }
#endif
    if (pend >= 0) face_commit<FST, false>(s_face, pend, xp, yp, near, far, delta, depth_min, best);
}

// Which of the bin's sixteen 8x8 pixel blocks a staged face may touch: bit 4 r + j (block column j, row
// r of the 32x32 bin at (bx0, by0)) is set when the face's float bbox meets the block's pixel-centre
// extent [pix_center(bx0 + 8 j), pix_center(bx0 + 8 j + 7)] x (the same in y) and, with CULL, its
// edges do not fail at every pixel centre of the block (nr_block_culled) -- the predicate each wave's
// ballot used to evaluate per 8x8 block and 64 staged faces, with the same float operations, so the
// walked faces are the same.  Evaluated once per staged face, by its staging lane, which takes its
// face's overlapped blocks one at a time: the edge cull runs once per (face, overlapped block) pair
// instead of once per (wave, 64 staged faces), where most of the 64 lanes had no overlap to test.
template <bool CULL>
__device__ __forceinline__ uint32_t face_block_mask(float x0, float y0, float x1, float y1, float x2, float y2,
                                                    float xmin, float xmax, float ymin, float ymax,
                                                    const float* __restrict__ ext, int r0, int nr) {
    // ext: the blocks' pixel-centre extents, [0..3] x lo, [4..7] x hi, [8..11] y lo, [12..15] y hi per
    // block column / row (block_extents, in LDS: computed once per bin, read as broadcasts); only the
    // block rows r0 .. r0 + nr - 1 are evaluated (the deep variant splits a face's rows over two lanes)
    uint32_t mx = 0, m = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) mx |= (!(ext[4 + j] < xmin || ext[j] > xmax) ? 1u : 0u) << j;
#pragma unroll
    for (int r = 0; r < 4; r++)
        if (r >= r0 && r < r0 + nr) m |= !(ext[12 + r] < ymin || ext[8 + r] > ymax) ? mx << (4 * r) : 0u;
    if (CULL) {
        const float A = x1 - x0, B = y1 - y0, C = x2 - x1, D = y2 - y1, E = x0 - x2, F = y0 - y2;
        for (uint32_t rest = m; rest; rest &= rest - 1) {
            const int u = __builtin_ctz(rest), j = u & 3, r = u >> 2;
            const float xl = ext[j], xh = ext[4 + j], yl = ext[8 + r], yh = ext[12 + r];
            if (nr_block_culled(x0, y0, x1, y1, x2, y2, A, B, C, D, E, F, 0.5f * (xl + xh), 0.5f * (yl + yh),
                                0.5f * (xh - xl), 0.5f * (yh - yl)))
                m &= ~(1u << u);
        }
    }
    return m;
}
// thread t < 16 of the block writes extent t of the bin's 8x8 blocks (face_block_mask's table)
__device__ __forceinline__ void block_extents(float* ext, int t, int bx0, int by0, int S) {
    if (t < 16) {
        const int base = (t & 8) ? by0 : bx0, j = t & 3;
        ext[t] = pix_center(base + 8 * j + ((t & 4) ? 7 : 0), S);
    }
}

// The bin's 64 4x4 quarters (quarter q = 8 R + J: column J, row R), for the dealt-quarter deep walk:
// thread t < 32 writes extent t ([0..7] x lo, [8..15] x hi, [16..23] y lo, [24..31] y hi per quarter
// column / row), and face_quarter_mask gives quarter rows r0 .. r0 + 3 of a face's mask (bit
// 8 (R - r0) + J): the bbox test and, with CULL, the edge cull (nr_block_culled, exact for any
// rectangle of pixel centres), as face_block_mask does for the 8x8 blocks
__device__ __forceinline__ void quarter_extents(float* ext4, int t, int bx0, int by0, int S) {
    if (t < 32) {
        const int base = (t & 16) ? by0 : bx0, j = t & 7;
        ext4[t] = pix_center(base + 4 * j + ((t & 8) ? 3 : 0), S);
    }
}
template <bool CULL>
__device__ __forceinline__ uint32_t face_quarter_mask(const float* __restrict__ c, const float* __restrict__ ext4, int r0) {
    const float x0 = c[0], y0 = c[1], x1 = c[3], y1 = c[4], x2 = c[6], y2 = c[7];
    const float xmin = fminf(fminf(x0, x1), x2), xmax = fmaxf(fmaxf(x0, x1), x2);
    const float ymin = fminf(fminf(y0, y1), y2), ymax = fmaxf(fmaxf(y0, y1), y2);
    uint32_t mx = 0, m = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) mx |= (!(ext4[8 + j] < xmin || ext4[j] > xmax) ? 1u : 0u) << j;
#pragma unroll
    for (int r = 0; r < 4; r++) m |= !(ext4[24 + r0 + r] < ymin || ext4[16 + r0 + r] > ymax) ? mx << (8 * r) : 0u;
    // (the edge cull per quarter: culling per 8x8 block and spreading each block's bit over its
    // quarters halved the staging's culls, but the longer lists cost the torus forward more, 0.114 ->
    // 0.118 ms, gpurun_out/dq2)
    if (CULL) {
        const float A = x1 - x0, B = y1 - y0, C = x2 - x1, D = y2 - y1, E = x0 - x2, F = y0 - y2;
        for (uint32_t rest = m; rest; rest &= rest - 1) {
            const int bit = __builtin_ctz(rest), j = bit & 7, r = r0 + (bit >> 3);
            const float xl = ext4[j], xh = ext4[8 + j], yl = ext4[16 + r], yh = ext4[24 + r];
            if (nr_block_culled(x0, y0, x1, y1, x2, y2, A, B, C, D, E, F, 0.5f * (xl + xh), 0.5f * (yl + yh),
                                0.5f * (xh - xl), 0.5f * (yh - yl)))
                m &= ~(1u << bit);
        }
    }
    return m;
}

// stage staged-face slot `slot` of candidate face f (coordinates c) and its block mask.  half (the
// 1024-thread variant: twice as many threads as staged faces): thread `slot` evaluates the mask's
// block rows 0-1 and thread FST + slot rows 2-3 (stage_mask_rows), each writing its byte, so the edge
// culls of a round spread over every wave of the block.
template <int FST, bool CULL, bool MASK = true>
__device__ __forceinline__ void stage_face(float4* s_face, uint16_t* s_bm, int slot, const float* __restrict__ c, int f,
                                           const float* __restrict__ ext, bool half) {
    float4* e = s_face + slot;
    const float x0 = c[0], y0 = c[1], z0 = c[2], x1 = c[3], y1 = c[4], z1 = c[5];
    const float x2 = c[6], y2 = c[7], z2 = c[8];
    const float xmin = fminf(fminf(x0, x1), x2), xmax = fmaxf(fmaxf(x0, x1), x2);
    const float ymin = fminf(fminf(y0, y1), y2), ymax = fmaxf(fmaxf(y0, y1), y2);
    e[0 * FST] = make_float4(xmin, xmax, ymin, ymax);
    if (MASK) {
        const uint32_t m = face_block_mask<CULL>(x0, y0, x1, y1, x2, y2, xmin, xmax, ymin, ymax, ext, 0, half ? 2 : 4);
        if (half) reinterpret_cast<uint8_t*>(s_bm)[2 * slot] = (uint8_t)m;
        else s_bm[slot] = (uint16_t)m;
    }
    e[1 * FST] = make_float4(fminf(fminf(z0, z1), z2), x1 * y2 - x2 * y1, x0 * y1 - x1 * y0, x2 * y0 - x0 * y2);
    e[2 * FST] = make_float4(y0, y2, x0, x2);
    e[3 * FST] = make_float4(x1 - x0, x0 - x2, y1 - y0, y0 - y2);
    e[4 * FST] = make_float4(y1, x1, x2 - x1, y2 - y1);
    e[5 * FST] = make_float4(z0, z1, z2, __int_as_float(f));
    const bool ok = coord_ok(x0) && coord_ok(y0) && coord_ok(x1) && coord_ok(y1) && coord_ok(x2) && coord_ok(y2) &&
                    in_range(z0, 0x1p-20f, 0x1p20f) && in_range(z1, 0x1p-20f, 0x1p20f) &&
                    in_range(z2, 0x1p-20f, 0x1p20f);
    e[6 * FST] = make_float4(rcp_nr(z0), rcp_nr(z1), rcp_nr(z2), __int_as_float(ok ? 1 : 0));
}
template <bool CULL>
__device__ __forceinline__ void stage_mask_rows(uint16_t* s_bm, int slot, const float* __restrict__ c,
                                                const float* __restrict__ ext) {
    const float x0 = c[0], y0 = c[1], x1 = c[3], y1 = c[4], x2 = c[6], y2 = c[7];
    const float xmin = fminf(fminf(x0, x1), x2), xmax = fmaxf(fmaxf(x0, x1), x2);
    const float ymin = fminf(fminf(y0, y1), y2), ymax = fmaxf(fmaxf(y0, y1), y2);
    const uint32_t m = face_block_mask<CULL>(x0, y0, x1, y1, x2, y2, xmin, xmax, ymin, ymax, ext, 2, 2);
    reinterpret_cast<uint8_t*>(s_bm)[2 * slot + 1] = (uint8_t)(m >> 8);
}

// per-wave phase timestamps of the fused forward (timing builds only, tools/fwd_timing.py)
#ifdef NR_FWD_TIMING
constexpr long long NR_FTIMING_MAX = 1 << 22;
constexpr int NR_FTSLOTS = 10;  // per wave: 8 phase slots, then the wall clock (100 MHz, chip-wide) at start and end
__device__ unsigned long long g_fwd_t[NR_FTIMING_MAX];
// (k_raster_fwd only: a split forward's second launch, part 2, writes the upper half of the buffer, so
// the two launches' stamps do not overlap; tools/fwd_timing.py decodes each with its own block size)
#define NR_FTSTAMP(k, v)                                                                                   \
    do {                                                                                                   \
        const long long h_ = NR_FTIMING_MAX / 2;                                                           \
        const long long i_ = (((long long)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6)) * NR_FTSLOTS + (k); \
        const unsigned long long t_ = (v);                                                                 \
        if ((threadIdx.x & 63) == 0 && i_ < h_) g_fwd_t[i_ + (part == 2 ? h_ : 0)] = t_;                  \
    } while (0)
#else
#define NR_FTSTAMP(k, v) \
    do {                 \
    } while (0)
#endif

// 8 waves/SIMD (at v37 7 waves, with no spilled register, measured the same)
// (the 256-thread variant at 7 waves/SIMD: car forward +10 %, gpurun_out/e6)
constexpr int FWD_WPE = 8;
// SHADE (NTF == 256, anti-aliasing, no lights / backgrounds): the block also shades its bin's 16x16
// output pixels (k_shade's work, shade_quad) from the face ids it has just found, so the face-index
// map is not read back and k_shade has no launch of its own.
// CC (SHADE only): the channel count as a compile-time constant; CC = MAXC means rgb + sil + depth, 4
// rgb + sil (static_draw), so the epilogue's draw-flag tests and per-channel guards fold away (0: sh.C /
// sh.draw at run time)
// DQ (1024 threads): the dealt-quarter walk for bins of >= ZCULL_MIN candidates compiled in (its own
// instantiation: in the static-blocks kernel its registers and LDS cost the car's split deep launch
// 1.3 %, gpurun_out/dq3)
template <int NTF, bool SHADE, int CC = 0, bool DQ = false>
__global__ __launch_bounds__(NTF) __attribute__((amdgpu_waves_per_eu(FWD_WPE, 8))) void k_raster_fwd(const float* __restrict__ face_records, int rs,
                                                  const int2* __restrict__ bbox, const uint32_t* __restrict__ mask,
                                                  int F, Geom g, float near, float far, float delta,
                                                  int32_t* __restrict__ fim, Shade sh_in, float* __restrict__ images,
                                                  float* __restrict__ halo, uint8_t* __restrict__ binfg,
                                                  const int* __restrict__ order, int fim_sparse,
                                                  const int* __restrict__ split, int part,
                                                  const uint8_t* __restrict__ sg_parts) {
    using C = FwdCfg<NTF>;
    static_assert(!SHADE || ((NTF == 256 || NTF == 1024) && COARSE == 32), "fused shading: threads 0-255 shade a pixel each");
    constexpr int NSUB = C::NSUB, FCAP = C::FCAP, CAND = C::CAND;
    // the edge cull of staged faces per 8x8 block (face_block_mask).  Once a cost of ~40 VALU per wave
    // and 64 staged faces in every walk's ballot, which only the deep-bin variant paid back (headline
    // +2-5 %); evaluated once per (face, overlapped block) at staging since v56, it pays in every
    // variant (headline forward 0.1444 -> 0.1397 ms, torus 0.1207 -> 0.1181 ms, the car unchanged;
    // same-box A/B, 3 runs each, gpurun_out/e3)
    constexpr bool CULL = true;
    __shared__ __attribute__((aligned(16))) unsigned char s_raw[C::LDS_BASE + (DQ ? C::LDS_DQ : 0)];
    __shared__ int s_scan[C::NW];
    __shared__ int s_next;  // (dyn) next 8x8 block to walk
    float4* s_face = reinterpret_cast<float4*>(s_raw);
    int* s_cand = reinterpret_cast<int*>(s_raw + FCAP * FREC * 16);
    uint16_t* s_bm = reinterpret_cast<uint16_t*>(s_raw + FCAP * FREC * 16 + CAND * 4);  // staged faces' block masks
    float* s_ext = reinterpret_cast<float*>(s_raw + FCAP * FREC * 16 + CAND * 4 + FCAP * 2);  // block extents

    const int S = g.S;
    int b, bin_x, bin_y;
    bool known_empty = false;  // (ordered) the setup's counts say the bin has no candidate face
    int quad = -1;             // (part 3) this block walks one 16x16 quadrant of a deep bin
    if (order) {
        const int ob = ordered_bin<DQ>(order, split, part, g.B, g.nbins, g.nbx, b, bin_x, bin_y, quad);
        if (ob < 0) return;  // past this launch's part of the list (block-uniform, before any barrier)
        known_empty = ob == 1;
    } else {
        block_item_tile(g.group, g.nbx, g.nby, b, bin_x, bin_y);
    }
    const int bin = bin_y * g.nbx + bin_x;
    const int bx0 = bin_x * COARSE;
    const int by0 = bin_y * COARSE;
    const int t = threadIdx.x;
    const int lane = t & 63, wid = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform: block extents in SGPRs
    block_extents(s_ext, t, bx0, by0, S);  // read after the first barrier below

    const uint32_t* words = mask + ((long long)b * g.nbins + bin) * g.nwords;
    const float* frb = face_records + (long long)b * F * rs;
    int32_t* __restrict__ fimb = fim + (long long)b * S * S;

    NR_FTSTAMP(0, clock64());
    NR_FTSTAMP(8, wall_clock64());
#ifdef NR_FWD_TIMING
    unsigned long long t_stage = 0, t_wait = 0;  // staging rounds; (static blocks) waits after the walks
#endif
    // (DQ, sg_parts: sparse groups, a deep-first forward that does not split) the bin's mask words are
    // read through the list of the face groups with candidates in it, built here from the setup's
    // per-group counts (thread t: group t) by a block scan, ascending: virtual word v = 6 j + i is word
    // i of the j-th listed group, so the rounds below expand the same candidates in the same ascending
    // order while reading only the listed groups' words -- the only ones the setup wrote
    // (k_face_setup sparse_groups)
    constexpr int GW = SETUP_FACES / 32;
    __shared__ uint16_t s_gl[DQ ? NTF : 1];  // (the host takes this path only for <= NTF groups)
    bool sgm = false;   // (block-uniform)
    int nv = g.nwords;  // virtual words
    if (DQ && sg_parts && !known_empty) {
        const int groups = setup_groups(g);
        const int c = t < groups ? sg_parts[((long long)b * groups + t) * g.nbins + bin] : 0;
        int ng;
        const int o = block_scan<C::NW>(c ? 1 : 0, ng, s_scan);
        if (c) s_gl[o] = (uint16_t)t;
        __syncthreads();
        sgm = true;
        nv = ng * GW;
    }
    // virtual word v's bits, and its word index (wr) in the bin's mask row
    auto word_at = [&](int v, int& wr) -> uint32_t {
        if (DQ && sgm) {
            if (v >= nv) {
                wr = 0;
                return 0u;
            }
            const int j = v / GW;
            wr = (int)s_gl[j] * GW + (v - j * GW);
            return wr < g.nwords ? words[wr] : 0u;
        }
        wr = v;
        return v < g.nwords ? words[v] : 0u;
    };
    // the first round of mask words and its candidate count
    int wr0 = t;
    const uint32_t bits0 = !known_empty ? word_at(t, wr0) : 0u;
    // (256-thread variant, NTF < nwords <= 2 NTF, e.g. the car's shallow bins in a split forward) the
    // second round of words too, scanned in the same block scan (two 16-bit counts per thread), so a
    // bin whose candidates fit one staging round takes the dealt-block path
    constexpr bool TWO = NTF < 1024;
    const bool two = TWO && !known_empty && g.nwords > NTF && g.nwords <= 2 * NTF;
    const uint32_t bits1 = (two && t + NTF < g.nwords) ? words[t + NTF] : 0u;
    int total0 = 0, total1 = 0, off1 = 0;
    int off0 = 0;
    if (!known_empty) {
        int tot;
        const int off = block_scan<C::NW>(__builtin_popcount(bits0) | (__builtin_popcount(bits1) << 16), tot, s_scan);
        off0 = off & 0xffff;
        total0 = tot & 0xffff;
        off1 = off >> 16;
        total1 = tot >> 16;
    }
    NR_FTSTAMP(1, clock64());
    // one staging round holds every candidate of the bin (the usual case): the waves take the 16 8x8
    // blocks one at a time from a counter, so a wave that meets few faces goes on to another block
    // instead of idling at the block's end (static quadrants keep 80 % of the waves' time busy on the
    // headline, dealt blocks ~92 %, CPU-counted; measured fwd 0.212 -> 0.208 ms)
    // (not with 16 waves: one block each already; measured 0.824 -> 0.918 ms on the car)
    // (a known-empty bin takes this path too: it only writes its empty outputs)
    const bool dyn = known_empty || (NTF < 1024 && (g.nwords <= NTF || two) && total0 + total1 <= FCAP);
    int ncand = 0;  // the bin's candidate faces (block-uniform)
    unsigned short* s_slot = reinterpret_cast<unsigned short*>(s_cand);  // (dyn, SHADE) winners' staging slots
    static_assert(!SHADE || CAND * 4 >= COARSE * COARSE * 2, "slot map in the candidate list's space");
    if (dyn) {
        ncand = total0 + total1;
        if (ncand == 0) {
            for (int u = wid; u < 16 && !fim_sparse; u += C::NW) {
                const int px = bx0 + (u & 3) * 8 + (lane & 7), py = by0 + (u >> 2) * 8 + (lane >> 3);
                if (px < S && py < S) fimb[(int)__umul24(py, S) + px] = -1;
            }
        } else {
            int r = off0;
            for (uint32_t m = bits0; m; m &= m - 1, r++) s_cand[r] = t * 32 + __builtin_ctz(m);
            r = total0 + off1;
            for (uint32_t m = bits1; m; m &= m - 1, r++) s_cand[r] = (t + NTF) * 32 + __builtin_ctz(m);
            if (t == 0) s_next = 0;
            __syncthreads();
#ifdef NR_FWD_TIMING
            const unsigned long long ts0_ = clock64();
#endif
            // (one thread per face: splitting the masks of rounds of at most 128 faces over the idle
            // threads measured the same, and spilled a register, gpurun_out/e6)
            if (t < ncand) {
                const int f = s_cand[t];
                stage_face<FCAP, CULL>(s_face, s_bm, t, frb + f * rs, f, s_ext, false);
            }
            __syncthreads();
#ifdef NR_FWD_TIMING
            t_stage += clock64() - ts0_;
#endif
            for (;;) {
                int u = 0;
                if (lane == 0) u = atomicAdd(&s_next, 1);
                u = __builtin_amdgcn_readfirstlane(u);  // lane 0's value: the wave is whole here
                if (u >= 16) break;
                const int ox = (u & 3) * 8, oy = (u >> 2) * 8;
                float depth_min = far;
                int best = -1;
                // the block's pixel-centre extent: lanes 0 / 7 hold its first / last column, lanes
                // 0 / 56 its first / last row (read into SGPRs, no recomputation)
                const float xp = pix_center(bx0 + ox + (lane & 7), S), yp = pix_center(by0 + oy + (lane >> 3), S);
                walk_block<FCAP, SHADE>(s_face, s_bm, u, ncand, lane, xp, yp, near, far, delta, depth_min, best);
                int id = best;
                if (SHADE) {  // best is the staging slot: its face id is in the record's row 5
                    id = best >= 0 ? __float_as_int(s_face[5 * FCAP + best].w) : -1;
                    s_slot[(oy + (lane >> 3)) * COARSE + ox + (lane & 7)] = best >= 0 ? (unsigned short)best : 0xffff;
                }
                const int px = bx0 + ox + (lane & 7), py = by0 + oy + (lane >> 3);
                if (px < S && py < S) fimb[(int)__umul24(py, S) + px] = id;
            }
        }
    } else if (DQ && NTF >= 1024 && CULL && (total0 >= ZCULL_MIN || quad >= 0)) {
        // dealt quarters (the deep bins of the 1024-thread variant): in each staging round the bin's 64
        // 4x4 quarters, longest face list first, are dealt to the 16 waves from a counter; a wave walks
        // one quarter at a time on lanes 0-15, its pixels' state (depth, winner) in LDS between rounds.
        // With one 8x8 block per wave for the whole bin, the waves of the car's deep bins spent 65 % of
        // their walk phase waiting at each round's barrier for the round's heaviest block (timing build,
        // profiles/r05_v59_car_fwd_wave_phases.txt: walk 130k, wait 249k cycles per wave); dealt
        // quarters cut a round's span to 0.61x of the heaviest block's walk (CPU model of the car's
        // deep bins: the quarters' lists are 0.45x a block's, and the waves share them out).  They walk
        // ~1.8x the face-quarter pairs, though, and stage 64 quarter masks per face: in the split
        // forward's deep launch (part 1, the car) the deep bins then ended at 378 instead of 435 us but
        // took wave slots from the concurrent rest launch, which ended 27 us later (forward 0.442 ->
        // 0.446-0.454 ms); where the deep bins have the chip to themselves (one item: the 50k torus)
        // the forward went 0.134 -> 0.114 ms (gpurun_out/dq, dq2)
        constexpr int QD = C::LDS_BASE;
        uint64_t* s_q = reinterpret_cast<uint64_t*>(s_raw + QD);                       // staged faces' quarter masks
        float* s_ext4 = reinterpret_cast<float*>(s_raw + QD + FCAP * 8);              // quarter extents
        float* s_dm = reinterpret_cast<float*>(s_raw + QD + FCAP * 8 + 128);          // per-pixel depth (py 32 + px)
        int* s_best = reinterpret_cast<int*>(s_raw + QD + FCAP * 8 + 128 + COARSE * COARSE * 4);
        int* s_qc = s_best + COARSE * COARSE;                                          // per-quarter walk lengths
        int* s_qord = s_qc + 64;                                                       // quarters, longest first
        s_dm[t] = far;
        s_best[t] = -1;
        quarter_extents(s_ext4, t, bx0, by0, S);
        // a quadrant block (quad >= 0) keeps only its quadrant's 16 quarters in the staged masks
        // (quarter q = 8 R + J: J < 4 in the left half, R < 4 in the top half), so the faces that miss
        // the quadrant are never walked and the other quarters' lengths are 0 (never dealt); it stages
        // every candidate as the whole-bin block does, and computes only its half of the mask rows
        const uint64_t qkeep = quad < 0 ? ~0ull
                                        : ((quad & 1) ? 0xF0F0F0F0F0F0F0F0ull : 0x0F0F0F0F0F0F0F0Full) &
                                              ((quad & 2) ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull);
        const bool rows_lo = quad < 0 || !(quad & 2), rows_hi = quad < 0 || (quad & 2);
        uint32_t bits = bits0;
        int total = total0, off = off0, w = wr0;
        for (int wbase = 0;;) {
            ncand += total;
            for (int cbase = 0; cbase < total; cbase += CAND) {
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
#ifdef NR_FWD_TIMING
                    const unsigned long long ts0_ = clock64();
#endif
                    // records by threads 0 .. n-1 with quarter rows 0-3 of the masks, rows 4-7 by
                    // threads FCAP .. FCAP + n - 1
                    if (t < n) {
                        const float* c = frb + s_cand[j0 + t] * rs;
                        stage_face<FCAP, CULL, false>(s_face, nullptr, t, c, s_cand[j0 + t], nullptr, false);
                        reinterpret_cast<uint32_t*>(s_q)[2 * t] =
                            rows_lo ? face_quarter_mask<CULL>(c, s_ext4, 0) & (uint32_t)qkeep : 0u;
                    } else if (t >= FCAP && t - FCAP < n) {
                        reinterpret_cast<uint32_t*>(s_q)[2 * (t - FCAP) + 1] =
                            rows_hi ? face_quarter_mask<CULL>(frb + s_cand[j0 + t - FCAP] * rs, s_ext4, 4) &
                                          (uint32_t)(qkeep >> 32)
                                    : 0u;
                    }
                    if (t == 0) s_next = 0;
                    __syncthreads();
#ifdef NR_FWD_TIMING
                    t_stage += clock64() - ts0_;
#endif
                    {  // quarter lengths: wave w counts quarters 4 w .. 4 w + 3 over the staged faces
                        int cq[4] = {0, 0, 0, 0};
                        for (int c0 = 0; c0 < n; c0 += 64) {
                            const uint64_t m = c0 + lane < n ? s_q[c0 + lane] : 0ull;
#pragma unroll
                            for (int i = 0; i < 4; i++) cq[i] += __popcll(__ballot((m >> (4 * wid + i)) & 1ull));
                        }
                        if (lane < 4) s_qc[4 * wid + lane] = lane == 0 ? cq[0] : lane == 1 ? cq[1] : lane == 2 ? cq[2] : cq[3];
                    }
                    __syncthreads();
                    if (wid == 0) {  // longest first (ties by index): lane q's rank among the 64
                        const int mc = s_qc[lane];
                        int rank = 0;
                        for (int j = 0; j < 64; j++) {
                            const int oc = s_qc[j];
                            rank += (oc > mc || (oc == mc && j < lane)) ? 1 : 0;
                        }
                        s_qord[rank] = lane;
                    }
                    __syncthreads();
                    for (;;) {
                        int k = 0;
                        if (lane == 0) k = atomicAdd(&s_next, 1);
                        k = __builtin_amdgcn_readfirstlane(k);
                        if (k >= 64) break;
                        const int q = s_qord[k];
                        if (s_qc[q] == 0) break;  // (longest first: the rest are empty too)
                        const int px = (q & 7) * 4 + (lane & 3), py = (q >> 3) * 4 + ((lane >> 2) & 3);
                        const bool on = lane < 16;
                        const int pix = py * COARSE + px;
#ifndef NR_NO_W4
                        float dm = s_dm[pix];  // (lanes 16-63: copies of lanes 0-15, walk_quarter4)
#else
                        float dm = on ? s_dm[pix] : -INFINITY;  // lanes 16-63: no pixel (and no share of the wave's depth maximum)
#endif
                        int best = on ? s_best[pix] : -1;
                        const float xq = pix_center_div(bx0 + px, S), yq = pix_center_div(by0 + py, S);
#ifndef NR_NO_W4
                        walk_quarter4<FCAP>(s_face, s_q, q, n, lane, xq, yq, near, far, delta, dm, best);
#else
                        walk_block<FCAP, false, true, uint64_t, true>(s_face, s_q, q, n, lane, xq, yq, near, far, delta,
                                                                      dm, best);
#endif
                        if (on) {
                            s_dm[pix] = dm;
                            s_best[pix] = best;
                        }
                    }
#ifdef NR_FWD_TIMING
                    const unsigned long long tw0_ = clock64();
#endif
                    __syncthreads();
#ifdef NR_FWD_TIMING
                    t_wait += clock64() - tw0_;
#endif
                }
            }
            wbase += NTF;
            if (wbase >= nv) break;
            bits = word_at(wbase + t, w);
            off = block_scan<C::NW>(__builtin_popcount(bits), total, s_scan);
        }
        // thread t: pixel (t & 31, t >> 5) of the bin (a quadrant block: of its quadrant only)
        const int fbest = s_best[t];
        {
            const int px = bx0 + (t & 31), py = by0 + (t >> 5);
            const bool mine = quad < 0 || (((t >> 4) & 1) == (quad & 1) && ((t >> 9) & 1) == (quad >> 1));
            if (mine && px < S && py < S && (ncand > 0 || !fim_sparse)) fimb[(int)__umul24(py, S) + px] = fbest;
        }
        if (SHADE && ncand > 0) {
            int* s_fim = reinterpret_cast<int*>(s_raw);
            __syncthreads();
            s_fim[t] = fbest;
        }
    } else {
        // static blocks: wave w walks its NSUB blocks; the per-pixel state stays in registers over
        // the staging rounds
        float xp[NSUB], yp[NSUB];
        float depth_min[NSUB];
        int best[NSUB];
        int ublk[NSUB];  // the 8x8 blocks' bits in the block masks
#pragma unroll
        for (int k = 0; k < NSUB; k++) {
            int ox, oy;
            C::block_of(wid, k, ox, oy);
            xp[k] = pix_center_div(bx0 + ox + (lane & 7), S);
            yp[k] = pix_center_div(by0 + oy + (lane >> 3), S);
            ublk[k] = (oy >> 3) * 4 + (ox >> 3);
            depth_min[k] = far;
            best[k] = -1;
        }
        uint32_t bits = bits0;
        int total = total0, off = off0, w = wr0;
        for (int wbase = 0;;) {
            ncand += total;
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
#ifdef NR_FWD_TIMING
                    const unsigned long long ts0_ = clock64();
#endif
                    constexpr bool half = NTF >= 2 * FCAP;  // the 1024-thread variant
                    if (t < n) {
                        const int f = s_cand[j0 + t];
                        stage_face<FCAP, CULL>(s_face, s_bm, t, frb + f * rs, f, s_ext, half);
                    } else if (half && t >= NTF / 2 && t - NTF / 2 < n) {
                        stage_mask_rows<CULL>(s_bm, t - NTF / 2, frb + s_cand[j0 + t - NTF / 2] * rs, s_ext);
                    }
                    __syncthreads();
#ifdef NR_FWD_TIMING
                    t_stage += clock64() - ts0_;  // staging rounds (the expansion is in the walk's share)
#endif
                    if (CULL && total0 >= ZCULL_MIN) {  // (a separate instantiation: the plain walk's code unchanged)
#pragma unroll
                        for (int k = 0; k < NSUB; k++)
                            walk_block<FCAP, false, true>(s_face, s_bm, ublk[k], n, lane, xp[k], yp[k], near, far, delta,
                                                          depth_min[k], best[k]);
                    } else {
#pragma unroll
                        for (int k = 0; k < NSUB; k++)
                            walk_block<FCAP, false>(s_face, s_bm, ublk[k], n, lane, xp[k], yp[k], near, far, delta,
                                                    depth_min[k], best[k]);
                    }
#ifdef NR_FWD_TIMING
                    const unsigned long long tw0_ = clock64();
#endif
                    __syncthreads();
#ifdef NR_FWD_TIMING
                    t_wait += clock64() - tw0_;
#endif
                }
            }
            wbase += NTF;
            if (wbase >= nv) break;
            bits = word_at(wbase + t, w);
            off = block_scan<C::NW>(__builtin_popcount(bits), total, s_scan);
        }
#pragma unroll
        for (int k = 0; k < NSUB; k++) {
            int ox, oy;
            C::block_of(wid, k, ox, oy);
            const int px = bx0 + ox + (lane & 7), py = by0 + oy + (lane >> 3);
            if (px < S && py < S && (ncand > 0 || !fim_sparse)) fimb[(int)__umul24(py, S) + px] = best[k];
        }
        if (SHADE && ncand > 0) {
            // the bin's 32x32 face ids go through LDS (the staging area is free once every wave has walked)
            int* s_fim = reinterpret_cast<int*>(s_raw);
            __syncthreads();
#pragma unroll
            for (int k = 0; k < NSUB; k++) {
                int ox, oy;
                C::block_of(wid, k, ox, oy);
                s_fim[(oy + (lane >> 3)) * COARSE + ox + (lane & 7)] = best[k];
            }
        }
    }

    NR_FTSTAMP(3, clock64());
    NR_FTSTAMP(2, t_stage);
    NR_FTSTAMP(7, t_wait);
    // may the bin hold a foreground pixel (the backward skips its tiles when not): a bin without
    // candidate faces holds none
    if (binfg && t == 0) binfg[(long long)b * g.nbins + bin] = ncand > 0 ? 1 : 0;
    if (!SHADE) {
        NR_FTSTAMP(4, clock64());
        NR_FTSTAMP(5, clock64());
        NR_FTSTAMP(9, wall_clock64());
        NR_FTSTAMP(6, (unsigned long long)ncand);
    }
    if (SHADE && ncand == 0) {
        // an empty bin: every channel of its output pixels is 0 (sil, depth and rgb of background;
        // no backgrounds in this variant), as is every halo value.  With the bin flags the halo values
        // are not written: the backward reads a halo pixel of a flagged-empty bin as 0
        Shade sh = sh_in;
        if (CC) {
            sh.C = CC;
            sh.draw = static_draw(CC);
        }
        const int m = t >> 4, n = t & 15;
        const int iy = by0 + 2 * m, ix = bx0 + 2 * n;
        if ((NTF == 256 || t < 256) && iy + 1 < S && ix + 1 < S) shade_quad_empty(sh, b, S, iy, ix, images, binfg ? nullptr : halo);
        NR_FTSTAMP(4, clock64());
        NR_FTSTAMP(5, clock64());
        NR_FTSTAMP(9, wall_clock64());
        NR_FTSTAMP(6, 0ull);
        return;
    }
    if (SHADE) {
        // thread t shades the output pixel whose internal quad is (2 (t >> 4), 2 (t & 15)), from the
        // face ids in LDS (dyn: the winners' staging slots)
        Shade sh = sh_in;
        sh.nl = 0;
        sh.bg = nullptr;
        if (CC) {
            sh.C = CC;
            sh.draw = static_draw(CC);
        }
        __syncthreads();
        NR_FTSTAMP(4, clock64());
        const int m = t >> 4, n = t & 15;
        const int iy = by0 + 2 * m, ix = bx0 + 2 * n;
        // (a quadrant block shades its quadrant's 8x8 output pixels)
        const bool qmine = quad < 0 || ((n >> 3) == (quad & 1) && (m >> 3) == (quad >> 1));
        if ((NTF == 256 || t < 256) && qmine && iy + 1 < S && ix + 1 < S) {
            int fis[4];
            if (dyn) {
                const uint32_t q0 = *reinterpret_cast<const uint32_t*>(s_slot + (2 * m) * COARSE + 2 * n);      // d, b
                const uint32_t q1 = *reinterpret_cast<const uint32_t*>(s_slot + (2 * m + 1) * COARSE + 2 * n);  // c, a
                const uint32_t sl[4] = {q1 >> 16, q0 >> 16, q1 & 0xffff, q0 & 0xffff};
#pragma unroll
                for (int i = 0; i < 4; i++) fis[i] = sl[i] == 0xffff ? -1 : __float_as_int(s_face[5 * FCAP + sl[i]].w);
            } else {
                const int* s_fim = reinterpret_cast<const int*>(s_raw);
                const int2 q0 = *reinterpret_cast<const int2*>(s_fim + (2 * m) * COARSE + 2 * n);      // d, b
                const int2 q1 = *reinterpret_cast<const int2*>(s_fim + (2 * m + 1) * COARSE + 2 * n);  // c, a
                fis[0] = q1.y;
                fis[1] = q0.y;
                fis[2] = q1.x;
                fis[3] = q0.x;
            }
            shade_quad(sh, face_records + (long long)b * F * FACE_REC, b, S, iy, ix, fis, images, halo);
        }
        NR_FTSTAMP(5, clock64());
        NR_FTSTAMP(9, wall_clock64());
        NR_FTSTAMP(6, (unsigned long long)ncand);
    }
}


// textures [Bt, 3, H, W] (any strides) -> RGBA rows [Bt, HWp, 4] (alpha slot 0), read by the sampling
__global__ void k_tex_pack(TexPack pk) {  // standalone form (no face setup to carry it)
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < pk.n) tex_pack_one(pk, i);
}

}  // namespace
