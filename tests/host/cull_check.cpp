// Host check of the forward's edge cull (csrc/nr_cull.h, built with g++ -ffp-contract=off): for
// random triangles and 8x8 pixel blocks, a culled block must fail the reference's edge tests
// (.cu:107-116, as face_pass evaluates them in float) at every one of its 64 pixel centres.
// Triangle kinds: random, snapped to pixel centres with an axis-aligned edge 1-2 (c2 exactly 0 on
// its line), tiny, degenerate (collinear / repeated corners), huge and non-finite coordinates.
// Prints "checked N culled M passes-in-culled 0"; exits 1 on a violation.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "nr_cull.h"

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint32_t next() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)(rng >> 11);
}
static float unif(float lo, float hi) { return lo + (hi - lo) * (float)((next() & 0xffffff) / 16777216.0); }
static float pc(int i, int S) { return (float)((2. * i + 1 - S) / S); }

int main(int argc, char** argv) {
    const long trials = argc > 1 ? atol(argv[1]) : 400000;
    const int sizes[4] = {64, 96, 512, 1000};
    long culled = 0, bad = 0;
    for (long t = 0; t < trials; t++) {
        const int S = sizes[next() % 4];
        const int bx = (int)(next() % (unsigned)(S / 8)) * 8, by = (int)(next() % (unsigned)(S / 8)) * 8;
        float x[3], y[3];
        const int kind = next() % 6;
        const int cx = bx + (int)(next() % 24) - 8, cy = by + (int)(next() % 24) - 8;
        for (int k = 0; k < 3; k++) {
            if (kind == 0) {  // random, within a few blocks
                x[k] = pc(cx, S) + unif(-40.f, 40.f) / S;
                y[k] = pc(cy, S) + unif(-40.f, 40.f) / S;
            } else if (kind == 1 || kind == 2) {  // snapped to pixel centres
                x[k] = pc(cx + (int)(next() % 25) - 12, S);
                y[k] = pc(cy + (int)(next() % 25) - 12, S);
            } else if (kind == 3) {  // tiny
                x[k] = pc(cx, S) + unif(-2.f, 2.f) / S;
                y[k] = pc(cy, S) + unif(-2.f, 2.f) / S;
            } else if (kind == 4) {  // degenerate: on one line through corner 0
                const float dx = unif(-20.f, 20.f) / S, dy = unif(-20.f, 20.f) / S;
                const float s = k == 0 ? 0.f : (float)(int)(next() % 5) - 2.f;
                x[k] = pc(cx, S) + s * dx;
                y[k] = pc(cy, S) + s * dy;
            } else {  // huge / non-finite corners now and then
                x[k] = pc(cx, S) + unif(-40.f, 40.f) / S;
                y[k] = pc(cy, S) + unif(-40.f, 40.f) / S;
                const uint32_t r = next() % 16;
                if (r == 0) x[k] = INFINITY;
                if (r == 1) y[k] = -INFINITY;
                if (r == 2) x[k] = NAN;
                if (r == 3) y[k] = 1e30f;
                if (r == 4) x[k] = -3e38f;
            }
        }
        if (kind == 1) y[2] = y[1];  // edge 1-2 horizontal: c2 == 0 along a pixel row
        if (kind == 2) x[2] = x[1];  // or vertical
        // the staged differences (stage_face)
        const float A = x[1] - x[0], B = y[1] - y[0], C = x[2] - x[1], D = y[2] - y[1], E = x[0] - x[2], F = y[0] - y[2];
        const float xl = pc(bx, S), xh = pc(bx + 7, S), yl = pc(by, S), yh = pc(by + 7, S);
        if (!nr_block_culled(x[0], y[0], x[1], y[1], x[2], y[2], A, B, C, D, E, F, 0.5f * (xl + xh), 0.5f * (yl + yh),
                             0.5f * (xh - xl), 0.5f * (yh - yl)))
            continue;
        culled++;
        for (int j = 0; j < 8; j++) {
            for (int i = 0; i < 8; i++) {
                const float xp = pc(bx + i, S), yp = pc(by + j, S);
                const float c1 = (yp - y[0]) * A - B * (xp - x[0]);
                const float c2 = (yp - y[1]) * C - D * (xp - x[1]);
                const float c3 = (yp - y[2]) * E - F * (xp - x[2]);
                if (!(c1 * c2 < 0) && !(c2 * c3 < 0)) {
                    if (bad < 5)
                        fprintf(stderr, "violation: S %d block (%d,%d) px (%d,%d) kind %d tri (%a,%a) (%a,%a) (%a,%a)\n", S, bx,
                                by, i, j, kind, x[0], y[0], x[1], y[1], x[2], y[2]);
                    bad++;
                }
            }
        }
    }
    printf("checked %ld culled %ld passes-in-culled %ld\n", trials, culled, bad);
    return bad ? 1 : 0;
}
