// fracenc_color.hip — the frame loader's colour conversion on the device
// (ImageIO::rgb2yuv, image/ImageIO.cpp:11-13,43-58).
//
//   Y(x, y)          = clamp(fma(0.114, b, fma(0.299, r, 0.587·g)))            every pixel
//   U(i, j), V(i, j) = the same form with the U / V weights, + 128, of pixel (2i+1, 2j+1)
//
// The reference writes chroma from every pixel of a 2×2 quad to (x/2, y/2), so the
// odd pixel (the last writer) wins; only that pixel is converted here.  The fused
// form is the built reference's (GCC contracts the first product into the first
// addition under -mfma), pinned on all 2^24 colours against oracle/_ref.
// clamp() truncates toward zero after the range checks (ImageIO.cpp:11-13).
//
// HBM-bound byte work: 3 B read + 1.5 B written per pixel.  rgb2yuv_quads4 gives
// each lane a 4-column × 2-row block (three aligned dword loads per row, one dword
// Y store per row, one u16 store per chroma plane); rgb2yuv_generic covers any
// alignment / odd size, one lane per 2×2 quad.
#include "fracenc_common.h"

namespace fracenc {

struct ColorArgs {
    const uint8_t* rgb;
    uint32_t w, h, rgb_stride;
    uint8_t* y;
    uint32_t ys;
    uint8_t* u;
    uint32_t us;
    uint8_t* v;
    uint32_t vs;
};

__device__ inline uint8_t clamp_u8(double x) { return x < 0.0 ? 0 : x > 255 ? 255 : (uint8_t)x; }

__device__ inline uint8_t luma(double r, double g, double b) { return clamp_u8(__fma_rn(0.114, b, __fma_rn(0.299, r, 0.587 * g))); }
__device__ inline uint8_t chroma_u(double r, double g, double b)
{
    return clamp_u8(__fma_rn(0.499, b, __fma_rn(-0.169, r, -0.331 * g)) + 128.0);
}
__device__ inline uint8_t chroma_v(double r, double g, double b)
{
    return clamp_u8(__fma_rn(-0.0813, b, __fma_rn(0.499, r, -0.418 * g)) + 128.0);
}

// One lane per 2×2 quad (any alignment; odd trailing row / column handled).
__global__ void __launch_bounds__(256) rgb2yuv_generic(ColorArgs a)
{
    const uint32_t qw = (a.w + 1) / 2, qh = (a.h + 1) / 2;
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (size_t)qw * qh)
        return;
    const uint32_t qx = (uint32_t)(q % qw), qy = (uint32_t)(q / qw);
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const uint32_t y = 2 * qy + dy;
        if (y >= a.h)
            break;
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
            const uint32_t x = 2 * qx + dx;
            if (x >= a.w)
                break;
            const uint8_t* p = a.rgb + (size_t)y * a.rgb_stride + 3 * (size_t)x;
            const double r = p[0], g = p[1], b = p[2];
            a.y[(size_t)y * a.ys + x] = luma(r, g, b);
            if (dx == 1 && dy == 1 && qx < a.w / 2 && qy < a.h / 2) {
                a.u[(size_t)qy * a.us + qx] = chroma_u(r, g, b);
                a.v[(size_t)qy * a.vs + qx] = chroma_v(r, g, b);
            }
        }
    }
}

// Fast path: w % 4 == 0, h even, rgb_stride / ys % 4 == 0, us / vs % 2 == 0, pointers aligned.
// Lane (bx, by) converts columns [4bx, 4bx+4) of rows 2by, 2by+1.
__global__ void __launch_bounds__(256) rgb2yuv_quads4(ColorArgs a)
{
    const uint32_t bw = a.w / 4, bh = a.h / 2;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)bw * bh)
        return;
    const uint32_t bx = (uint32_t)(t % bw), by = (uint32_t)(t / bw);
    uint32_t oddu = 0, oddv = 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const uint32_t y = 2 * by + dy;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.rgb + (size_t)y * a.rgb_stride + 12 * (size_t)bx);
        const uint32_t w0 = __builtin_nontemporal_load(src), w1 = __builtin_nontemporal_load(src + 1),
                       w2 = __builtin_nontemporal_load(src + 2);
        // bytes: r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
        const uint32_t px[4][3] = {{w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u},
                                   {w0 >> 24, w1 & 255u, (w1 >> 8) & 255u},
                                   {(w1 >> 16) & 255u, w1 >> 24, w2 & 255u},
                                   {(w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24}};
        uint32_t yw = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            yw |= (uint32_t)luma(px[k][0], px[k][1], px[k][2]) << (8 * k);
        *reinterpret_cast<uint32_t*>(a.y + (size_t)y * a.ys + 4 * (size_t)bx) = yw;
        if (dy == 1) {
#pragma unroll
            for (int k = 1; k < 4; k += 2) {
                oddu |= (uint32_t)chroma_u(px[k][0], px[k][1], px[k][2]) << (4 * (k - 1));
                oddv |= (uint32_t)chroma_v(px[k][0], px[k][1], px[k][2]) << (4 * (k - 1));
            }
        }
    }
    *reinterpret_cast<uint16_t*>(a.u + (size_t)by * a.us + 2 * (size_t)bx) = (uint16_t)oddu;
    *reinterpret_cast<uint16_t*>(a.v + (size_t)by * a.vs + 2 * (size_t)bx) = (uint16_t)oddv;
}

inline bool color_fast_path(const ColorArgs& a)
{
    auto al = [](const void* p, uintptr_t n) { return (reinterpret_cast<uintptr_t>(p) % n) == 0; };
    return a.w % 4 == 0 && a.h % 2 == 0 && a.rgb_stride % 4 == 0 && a.ys % 4 == 0 && a.us % 2 == 0 &&
           a.vs % 2 == 0 && al(a.rgb, 4) && al(a.y, 4) && al(a.u, 2) && al(a.v, 2);
}

} // namespace fracenc
