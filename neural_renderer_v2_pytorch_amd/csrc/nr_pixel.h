// Pixel centres of the reference without double arithmetic (shared by the kernels and the host
// check tests/host/pixel_centre_check.cpp, which compiles this header with g++).
#pragma once

#if defined(__HIPCC__)
#define NR_PX_HD __host__ __device__ __forceinline__
#else
#define NR_PX_HD inline
#endif

// rasterize_cuda_kernel.cu:76-77 computes (float)((2.0 * i + 1 - S) / S): a double division rounded
// to float.  The numerator 2 i + 1 - S and S are integers below 2^24 in magnitude, exact in float, so
// the IEEE single division of the two rounds to the same float (double rounding is innocuous for a
// quotient when the wider format carries at least 2 p + 2 bits: 53 >= 2 * 24 + 2).  The host check
// compares every (i, S) with S <= 16384 (the largest raster the library accepts) against the double
// formula, bit for bit.  The kernels evaluate this division with the exact shortened sequence
// (pix_center in nr_common.h: rcp_nr + div_nr, 8 VALU instructions without branches, where the
// double form is ~22 f64 instructions); tests/test_gpu_parity.py::test_pixel_centre_division
// checks that sequence against the IEEE division for every pixel centre of every such S.
NR_PX_HD float nr_pixel_centre(int i, int S) { return (float)(2 * i + 1 - S) / (float)S; }
