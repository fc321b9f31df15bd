// Micro-benchmark: what a grid of blocks that only read a flag byte and exit costs on gfx950.
// k_raster_bwd's grid has one block per 32x16 tile (32768 at the headline) and 64 % of them end at
// their bin's background flag; this times such a grid alone (LDS-sized like k_raster_bwd, 40 KB per
// block) against the same grid with no LDS, and a grid of fully live blocks for scale.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_empty_blocks.hip -o /tmp/ubench_empty
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int LDSB>
__global__ __launch_bounds__(256) void k_flag_exit(const unsigned char* __restrict__ flags, float* out, int n) {
    __shared__ float s[LDSB / 4 > 0 ? LDSB / 4 : 1];
    const int i = blockIdx.x;
    if (flags[i % n] == 0) return;
    s[threadIdx.x] = (float)i;
    __syncthreads();
    out[(long long)i * 256 + threadIdx.x] = s[255 - threadIdx.x];
}

int main() {
    const int nblk = 32768, nflags = 16384;
    unsigned char* flags;
    float* out;
    CHECK(hipMalloc(&flags, nflags));
    CHECK(hipMalloc(&out, (size_t)nblk * 256 * 4));
    CHECK(hipMemset(flags, 0, nflags));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 5; w++) launch();
        (void)hipEventRecord(e0);
        const int reps = 50;
        for (int r = 0; r < reps; r++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::printf("%-44s %8.2f us per launch\n", name, ms * 1e3f / reps);
    };
    run("32768 blocks, flag 0, 40 KB LDS", [&] { hipLaunchKernelGGL((k_flag_exit<40960>), dim3(nblk), dim3(256), 0, 0, flags, out, nflags); });
    run("32768 blocks, flag 0, no LDS", [&] { hipLaunchKernelGGL((k_flag_exit<0>), dim3(nblk), dim3(256), 0, 0, flags, out, nflags); });
    run("21000 blocks, flag 0, 40 KB LDS", [&] { hipLaunchKernelGGL((k_flag_exit<40960>), dim3(21000), dim3(256), 0, 0, flags, out, nflags); });
    run("1024 blocks, flag 0, 40 KB LDS", [&] { hipLaunchKernelGGL((k_flag_exit<40960>), dim3(1024), dim3(256), 0, 0, flags, out, nflags); });
    CHECK(hipMemset(flags, 1, nflags));
    run("32768 blocks, flag 1 (store 1 KB), 40 KB LDS", [&] { hipLaunchKernelGGL((k_flag_exit<40960>), dim3(nblk), dim3(256), 0, 0, flags, out, nflags); });
    CHECK(hipDeviceSynchronize());
    return 0;
}
