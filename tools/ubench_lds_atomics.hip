// Micro-benchmark: cost of LDS float atomic adds (ds_add_f32) by address-conflict degree, versus
// a DPP wave reduction.  Informs the backward kernel's accumulation design.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds_atomics.hip -o ubench && ./ubench
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int CONFLICT>
__global__ __launch_bounds__(256) void k_lds_add(float* out, int iters) {
    __shared__ float tab[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) tab[i] = 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    // lanes sharing one address: CONFLICT of them; spread over banks otherwise
    const int addr = ((lane / CONFLICT) * 33 + (threadIdx.x >> 6) * 512) & 4095;
    float v = 1.f + lane;
    for (int it = 0; it < iters; it++) {
        atomicAdd(&tab[(addr + it * 7) & 4095], v);
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = tab[0];
}

__device__ __forceinline__ float wave_sum(float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x111, 0xf, 0xf, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x112, 0xf, 0xf, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x114, 0xf, 0xf, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x118, 0xf, 0xf, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x142, 0xa, 0xf, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x143, 0xc, 0xf, false));
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}

__global__ __launch_bounds__(256) void k_dpp(float* out, int iters) {
    const int lane = threadIdx.x & 63;
    float v = 1.f + lane, acc = 0.f;
    for (int it = 0; it < iters; it++) {
        acc += wave_sum(v);
        v += 1.f;
    }
    if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = acc;
}

template <typename K>
float time_it(K k, float* out, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k<<<2048, 256>>>(out, iters);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) k<<<2048, 256>>>(out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    float* out;
    hipMalloc(&out, 2048 * 4 * sizeof(float));
    const int iters = 256;
    const double lane_ops = 2048.0 * 256 * iters;
    struct { const char* name; float ms; } r[] = {
        {"ds_add_f32 conflict 1 ", time_it(k_lds_add<1>, out, iters)},
        {"ds_add_f32 conflict 4 ", time_it(k_lds_add<4>, out, iters)},
        {"ds_add_f32 conflict 16", time_it(k_lds_add<16>, out, iters)},
        {"ds_add_f32 conflict 64", time_it(k_lds_add<64>, out, iters)},
        {"dpp wave_sum          ", time_it(k_dpp, out, iters)},
    };
    for (auto& x : r)
        printf("%s  %8.3f ms   %8.2f G lane-ops/s   %6.2f ns per wave-op per CU\n", x.name, x.ms,
               lane_ops / (x.ms * 1e-3) / 1e9, x.ms * 1e6 / (lane_ops / 64 / 256));
    hipFree(out);
    return 0;
}
