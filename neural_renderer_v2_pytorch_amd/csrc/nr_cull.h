// Edge cull of a face against a block of pixel centres (k_raster_fwd's deep-bin variant,
// NR_FWD_CULL). Plain float math, so the host check in tests/test_host.py compiles this same
// header with g++ and tests its exactness claim against the reference's per-pixel edge tests.
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define NR_HD __host__ __device__ __forceinline__
#else
#define NR_HD inline
#endif

// Sign of edge function c = (y - ay) A - B (x - ax) over the block [xc - hx, xc + hx] x
// [yc - hy, yc + hy]: c is affine in the pixel, so its range is centre +- hr. A sign is trusted when
// the whole range clears a margin covering the rounding of the reference's float evaluation and of
// this one: 2^-18 of the operand-magnitude bound T, at least 2^-60, so that a product of two trusted
// values cannot underflow to 0. NaN and infinite operands never give a trusted sign.
NR_HD void nr_edge_sign(float ax, float ay, float A, float B, float xc, float yc, float hx, float hy, bool& pos,
                        bool& neg) {
    const float dy = yc - ay, dx = xc - ax;
    const float cc = dy * A - B * dx;
    const float aA = fabsf(A), aB = fabsf(B);
    const float hr = hy * aA + hx * aB;
    const float T = (fabsf(yc) + fabsf(ay) + hy) * aA + (fabsf(xc) + fabsf(ax) + hx) * aB;
    const float m = fmaxf(T * 0x1p-18f, 0x1p-60f) + hr;
    pos = cc > m;
    neg = cc < -m;
}

// true only when the reference's edge tests (.cu:107-116: reject when c1 c2 < 0 or c2 c3 < 0) fail
// at every pixel centre of the block. (x_k, y_k): the corners; A..F the staged differences
// x1-x0, y1-y0, x2-x1, y2-y1, x0-x2, y0-y2. With c2 exactly 0 the reference passes a pixel whatever
// c1 and c3 are, so c1, c3 of opposite signs cull only with a trusted sign of c2.
NR_HD bool nr_block_culled(float x0, float y0, float x1, float y1, float x2, float y2, float A, float B, float C,
                           float D, float E, float F, float xc, float yc, float hx, float hy) {
    bool p1, n1, p2, n2, p3, n3;
    nr_edge_sign(x0, y0, A, B, xc, yc, hx, hy, p1, n1);
    nr_edge_sign(x1, y1, C, D, xc, yc, hx, hy, p2, n2);
    nr_edge_sign(x2, y2, E, F, xc, yc, hx, hy, p3, n3);
    return (p1 && n2) || (n1 && p2) || (p2 && n3) || (n2 && p3) || (((p1 && n3) || (n1 && p3)) && (p2 || n2));
}
