#include <hip/hip_runtime.h>
__device__ __forceinline__ float xor32(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    const int lane = threadIdx.x & 63;
    return __uint_as_float(lane < 32 ? r[1] : r[0]);
}
__device__ __forceinline__ float xor16(float x) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    const int lane = threadIdx.x & 63;
    return __uint_as_float(((lane >> 4) & 1) == 0 ? r[1] : r[0]);
}
__global__ void k(const float* a, float* o, float* o2) {
    int i = threadIdx.x;
    o[i] = xor32(a[i]);
    o2[i] = xor16(a[i]);
}
int main() {
    float *a, *o, *o2; hipMalloc(&a, 256); hipMalloc(&o, 256); hipMalloc(&o2, 256);
    float h[64]; for (int i = 0; i < 64; i++) h[i] = i;
    hipMemcpy(a, h, 256, hipMemcpyHostToDevice);
    k<<<1, 64>>>(a, o, o2);
    float r[64], r2[64]; hipMemcpy(r, o, 256, hipMemcpyDeviceToHost); hipMemcpy(r2, o2, 256, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 64; i++) { if (r[i] != (i ^ 32)) bad++; if (r2[i] != (i ^ 16)) bad++; }
    printf("bad=%d  r[0]=%g r[40]=%g r2[0]=%g r2[17]=%g\n", bad, r[0], r[40], r2[0], r2[17]);
    return bad != 0;
}
