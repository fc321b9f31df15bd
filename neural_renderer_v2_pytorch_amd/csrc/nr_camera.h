// nr_camera.h -- camera prologue (look_at + perspective) forward and backward kernels
// Part of nr_raster.hip (one translation unit); see that file and DESIGN.md.
#pragma once

#pragma clang fp contract(off)

namespace {

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

}  // namespace
