// Host check of csrc/nr_pixel.h (g++ -ffp-contract=off): nr_pixel_centre(i, S) equals the
// reference's pixel centre (float)((2.0 * i + 1 - S) / S) (rasterize_cuda_kernel.cu:76-77) bit for
// bit for every S in 1..16384 and every i in 0..S-1, plus a margin of indices outside the raster.
// Prints "checked N mismatches 0"; exits 1 on a mismatch.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nr_pixel.h"

static float reference(int i, int S) { return (float)((2. * i + 1 - S) / S); }

int main(int argc, char** argv) {
    const int smax = argc > 1 ? atoi(argv[1]) : 16384;
    long long checked = 0, bad = 0;
    for (int S = 1; S <= smax; S++) {
        for (int i = -2; i < S + 2; i++) {
            const float a = nr_pixel_centre(i, S), b = reference(i, S);
            uint32_t ua, ub;
            memcpy(&ua, &a, 4);
            memcpy(&ub, &b, 4);
            checked++;
            if (ua != ub) {
                if (bad < 5) printf("mismatch S=%d i=%d: %a vs %a\n", S, i, a, b);
                bad++;
            }
        }
    }
    printf("checked %lld mismatches %lld\n", checked, bad);
    return bad ? 1 : 0;
}
