/*
 * nr_oracle.c -- CPU restatement of the reference rasterizer's two native kernels.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP path; it is
 * never linked into, loaded by, or used as a fallback for the product library
 * (neural_renderer_v2_pytorch_amd/csrc).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.
 *
 * It restates, from the source text, the algorithm of
 *   /root/reference/neural_renderer_torch/cuda/rasterize_cuda_kernel.cu
 *     face_index_map_forward_safe_cuda_kernel   .cu:52-153  (launch .cu:362-390)
 *     compute_weight_map_cuda_kernel            .cu:246-308 (launch .cu:420-443)
 *     mask_foreground_{forward,backward}        .cu:7-49    (bound at rasterize_cuda.cpp:94-95, unused)
 * as plain C: one sequential brute-force scan of all faces per pixel, in ascending face
 * order, exactly as the reference kernel does.  OpenMP parallelises over pixels only.
 *
 * Numerics: must be compiled with -ffp-contract=off and
 * without -ffast-math; the double-precision pixel-centre formula and the double-literal
 * comparisons of the reference are reproduced literally.
 *
 * Pinning: tests/test_oracle_pins.py checks this restatement against the reference's own
 * fixtures (tests_torch/data/4e49873292196f02574b5684eaec43e9.png alpha channel and the
 * test_backward_case1 convergence scene) and against golden vectors produced by the
 * imported reference Python (tests/golden/make_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>

#define NR_EXPORT __attribute__((visibility("default")))

/* .cu:52-153 */
NR_EXPORT void oracle_face_index_map(const float* faces, int32_t* face_index, int batch_size,
                                     int num_faces, int image_size, float near, float far,
                                     int draw_backside, float eps, float depth_min_delta) {
    (void)eps; /* passed but unused by the reference kernel */
    const int is = image_size;
    const int nf = num_faces;
    const long long index_size = (long long)batch_size * is * is;
#pragma omp parallel for schedule(dynamic, 256)
    for (long long i = 0; i < index_size; i++) {
        const int bn = (int)(i / ((long long)is * is));
        const int pn = (int)(i % ((long long)is * is));
        const int yi = pn / is;
        const int xi = pn % is;
        const float yp = (float)((2. * yi + 1 - is) / is);
        const float xp = (float)((2. * xi + 1 - is) / is);

        const float* face = &faces[(size_t)bn * nf * 9];
        float depth_min = far;
        int face_index_min = -1;
        for (int fn = 0; fn < nf; fn++, face += 9) {
            const float x0 = face[0], y0 = face[1], z0 = face[2];
            const float x1 = face[3], y1 = face[4], z1 = face[5];
            const float x2 = face[6], y2 = face[7], z2 = face[8];

            if (xp < x0 && xp < x1 && xp < x2) continue;
            if (x0 < xp && x1 < xp && x2 < xp) continue;
            if (yp < y0 && yp < y1 && yp < y2) continue;
            if (y0 < yp && y1 < yp && y2 < yp) continue;

            if (!draw_backside) {
                if ((y2 - y0) * (x1 - x0) > (y1 - y0) * (x2 - x0)) continue;
            }

            const float c1 = (yp - y0) * (x1 - x0) - (y1 - y0) * (xp - x0);
            const float c2 = (yp - y1) * (x2 - x1) - (y2 - y1) * (xp - x1);
            if (c1 * c2 < 0) continue;
            const float c3 = (yp - y2) * (x0 - x2) - (y0 - y2) * (xp - x2);
            if (c2 * c3 < 0) continue;

            const float det = x2 * (y0 - y1) + x0 * (y1 - y2) + x1 * (y2 - y0);
            if ((double)fabsf(det) < 0.00000001) continue;

            if (depth_min < z0 && depth_min < z1 && depth_min < z2) continue;

            float w0 = yp * (x2 - x1) + xp * (y1 - y2) + (x1 * y2 - x2 * y1);
            float w1 = yp * (x0 - x2) + xp * (y2 - y0) + (x2 * y0 - x0 * y2);
            float w2 = yp * (x1 - x0) + xp * (y0 - y1) + (x0 * y1 - x1 * y0);
            const float w_sum = w0 + w1 + w2;
            w0 /= w_sum;
            w1 /= w_sum;
            w2 /= w_sum;

            const float zp = (float)(1. / (double)(w0 / z0 + w1 / z1 + w2 / z2));
            if (zp <= near || far <= zp) continue;

            if (zp <= depth_min - depth_min_delta) {
                depth_min = zp;
                face_index_min = fn;
            }
        }
        face_index[i] = face_index_min;
    }
}

/* .cu:246-308.  weight_map must be zero-initialised by the caller (rasterize.py:71). */
NR_EXPORT void oracle_weight_map(const float* faces, const int32_t* face_index_map, float* weight_map,
                                 int batch_size, int num_faces, int image_size) {
    const int is = image_size;
    const int nf = num_faces;
    const long long n = (long long)batch_size * is * is;
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < n; i++) {
        const int fi = face_index_map[i];
        if (fi < 0) continue;
        const int bn = (int)(i / ((long long)is * is));
        const int pn = (int)(i % ((long long)is * is));
        const int yi = pn / is;
        const int xi = pn % is;
        const float yp = (float)((2. * yi + 1 - is) / is);
        const float xp = (float)((2. * xi + 1 - is) / is);

        const float* face = &faces[((size_t)bn * nf + fi) * 9];
        const float x0 = face[0], y0 = face[1];
        const float x1 = face[3], y1 = face[4];
        const float x2 = face[6], y2 = face[7];

        float w[3];
        w[0] = yp * (x2 - x1) + xp * (y1 - y2) + (x1 * y2 - x2 * y1);
        w[1] = yp * (x0 - x2) + xp * (y2 - y0) + (x2 * y0 - x0 * y2);
        w[2] = yp * (x1 - x0) + xp * (y0 - y1) + (x0 * y1 - x1 * y0);
        float w_sum = w[0] + w[1] + w[2];
        if (w_sum < 0) {
            w[0] *= -1;
            w[1] *= -1;
            w[2] *= -1;
        }
        /* CUDA max(float, double) / min(float, double) resolve to fmax/fmin on double */
        w[0] = (float)fmax((double)w[0], 0.);
        w[1] = (float)fmax((double)w[1], 0.);
        w[2] = (float)fmax((double)w[2], 0.);
        w_sum = w[0] + w[1] + w[2];
        float* wm = &weight_map[i * 3];
        for (int j = 0; j < 3; j++) {
            w[j] /= w_sum;
            w[j] = (float)fmax(fmin((double)w[j], 1.), 0.);
            wm[j] = w[j];
        }
    }
}

/* .cu:7-27: copy `dim` floats of pixels whose face index is >= 0 */
NR_EXPORT void oracle_mask_foreground_forward(const int32_t* face_index, const float* data_in,
                                              float* data_out, long long n, int dim) {
    for (long long i = 0; i < n; i++)
        if (face_index[i] >= 0)
            for (int j = 0; j < dim; j++) data_out[i * dim + j] = data_in[i * dim + j];
}
