// fracenc_decode.hip — Decoder2 on the GPU (encode/Encoder2.hpp:67-99).
//
// Per iteration:
//   decode_apply   one wave per encode item: Frac::copy (encode/DecodeUtils.hpp:9-25) —
//                  target = clamp(trunc(fma(s, sample, o))) with SamplerBilinear::sample<double>
//                  of the source plane under the item's transform (image/sampler.h:21-38)
//   decode_rms     Σ (source − target)² over the plane (RootMeanSquare<Id> same-size branch,
//                  image/metrics.h:26-36), accumulated exactly in u64 (the reference's int32
//                  sum wraps; the host reproduces that from the exact sum)
// then the host compares rms with the epsilon and the source becomes a copy of the target.
#include "fracenc_common.h"

namespace fracenc {

struct DecodeArgs {
    const uint8_t* src;
    uint8_t* tgt;
    uint32_t stride;
    const frac_encode_item* items;
    uint32_t n;
};

// SamplerBilinear::sample's integer 2×2 sum at local (x, y) of `patch` under transform t
// (Transform::generateSampleOffsets, image/transform.h:96-109), with the edge clamp.
__device__ inline int sample_sum_dev(const uint8_t* __restrict__ img, uint32_t stride, uint32_t ox, uint32_t oy,
                                     uint32_t sw, uint32_t sh, uint32_t x, uint32_t y, int t)
{
    const Aff a = lut(t);
    if (x == sw - 1)
        --x;
    if (y == sh - 1)
        --y;
    const int64_t px = (int64_t)ox + a.a0 * (int64_t)x + a.a1 * (int64_t)y + a.a2 * ((int64_t)sw - 1) +
                       a.a3 * ((int64_t)sh - 1);
    const int64_t row = (int64_t)oy + a.a4 * (int64_t)x + a.a5 * (int64_t)y + a.a6 * ((int64_t)sw - 1) +
                        a.a7 * ((int64_t)sh - 1);
    const int64_t s = (int64_t)stride;
    const int64_t p0 = row * s + px;
    return (int)img[p0] + (int)img[p0 + a.a4 * s + a.a0] + (int)img[p0 + a.a5 * s + a.a1] +
           (int)img[p0 + (a.a4 + a.a5) * s + a.a0 + a.a1];
}

__global__ void __launch_bounds__(256) decode_apply(DecodeArgs a)
{
    const uint32_t it = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (it >= a.n)
        return;
    const frac_encode_item e = a.items[it];
    const uint32_t sw = e.match.sw, sh = e.match.sh;
    if (sw == 0 || sh == 0)
        return; // no eligible domain: the reference asserts here; the range is left untouched
    const double s = e.match.score.contrast, o = e.match.score.brightness;
    const int t = e.match.score.transform;
    for (uint32_t q = lane; q < e.w * e.h; q += 64) {
        const uint32_t x = q % e.w, y = q / e.w;
        const uint32_t sx = (x * sw) / e.w, sy = (y * sh) / e.h;
        const double smp = (double)sample_sum_dev(a.src, a.stride, e.match.x, e.match.y, sw, sh, sx, sy, t) / 4.0;
        const double v = __fma_rn(s, smp, o); // contrast * sample + brightness, FMA-contracted as built
        a.tgt[(size_t)(e.y + y) * a.stride + e.x + x] = v < 0.0 ? 0 : v > 255 ? 255 : (uint8_t)v;
    }
}

__global__ void __launch_bounds__(256) decode_rms(const uint8_t* __restrict__ src, const uint8_t* __restrict__ tgt,
                                                  uint32_t w, uint32_t h, uint32_t stride,
                                                  unsigned long long* __restrict__ sum)
{
    __shared__ unsigned long long part[4];
    unsigned long long acc = 0;
    const size_t total = (size_t)w * h;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t off = (i / w) * stride + (i % w);
        const int d = (int)src[off] - (int)tgt[off];
        acc += (unsigned long long)(d * d);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0)
        part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicAdd(sum, part[0] + part[1] + part[2] + part[3]);
}

// ---------------------------------------------------------------------------
// Fused form, used when the items tile the plane exactly (every pixel written once per
// iteration by an item with a domain): the rms of step i is Σ over the written pixels of
// (source − new target)², so it is accumulated while writing (per-block partial sums, no
// second pass), the source ← target copy becomes a buffer swap, and the convergence test
// (Encoder2.hpp:84-86, with the reference's int32 sum, metrics.h:27) runs on the device, so
// the host only checks a flag every few iterations.  After convergence the remaining
// enqueued iterations exit at their first instruction.
// ---------------------------------------------------------------------------
constexpr uint32_t kDecodeSlots = 256; // partial-sum slots between decode_fused and decode_check

struct DecodeState {
    int32_t done;       // 1 once rms < eps
    int32_t iterations; // Decoder2's returned count
    double rms;
};

__global__ void __launch_bounds__(256) decode_fused(DecodeArgs a, const DecodeState* __restrict__ st,
                                                    unsigned long long* __restrict__ partial)
{
    if (st->done)
        return;
    const uint32_t it = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    unsigned long long acc = 0;
    if (it < a.n) {
        const frac_encode_item e = a.items[it];
        const uint32_t sw = e.match.sw, sh = e.match.sh;
        const double s = e.match.score.contrast, o = e.match.score.brightness;
        const int t = e.match.score.transform;
        const bool pow2 = (e.w & (e.w - 1)) == 0, ratio2 = sw == 2 * e.w && sh == 2 * e.h;
        const uint32_t lw = e.w ? (uint32_t)__builtin_ctz(e.w) : 0u; // log2(e.w) when pow2
        for (uint32_t q = lane; q < e.w * e.h; q += 64) {
            const uint32_t x = pow2 ? q & (e.w - 1) : q % e.w, y = pow2 ? q >> lw : q / e.w;
            const uint32_t sx = ratio2 ? 2 * x : (x * sw) / e.w, sy = ratio2 ? 2 * y : (y * sh) / e.h;
            const double smp = (double)sample_sum_dev(a.src, a.stride, e.match.x, e.match.y, sw, sh, sx, sy, t) / 4.0;
            const double v = __fma_rn(s, smp, o);
            const uint8_t nv = v < 0.0 ? 0 : v > 255 ? 255 : (uint8_t)v;
            const size_t off = (size_t)(e.y + y) * a.stride + e.x + x;
            const int d = (int)a.src[off] - (int)nv;
            acc += (unsigned long long)(d * d);
            a.tgt[off] = nv;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        acc += __shfl_xor(acc, o, 64);
    __shared__ unsigned long long part[4];
    if (lane == 0)
        part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) // 256 accumulation slots: one load per thread in decode_check
        atomicAdd(&partial[blockIdx.x & (kDecodeSlots - 1)], part[0] + part[1] + part[2] + part[3]);
}

// one block: Σ of the kDecodeSlots partial slots (re-zeroed for the next step) → rms of step
// `step` exactly as the reference (int32 sum / area)
__global__ void __launch_bounds__(kDecodeSlots) decode_check(unsigned long long* __restrict__ partial,
                                                             uint64_t area, double eps, int32_t step,
                                                             int32_t last_step, DecodeState* __restrict__ st)
{
    if (st->done)
        return;
    unsigned long long acc = partial[threadIdx.x];
    partial[threadIdx.x] = 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        acc += __shfl_xor(acc, o, 64);
    __shared__ unsigned long long part[4];
    if ((threadIdx.x & 63) == 0)
        part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long sum = part[0] + part[1] + part[2] + part[3];
        const int32_t s32 = (int32_t)(uint32_t)(sum & 0xffffffffull);
        const double r = (double)s32 / (double)area;
        st->rms = r;
        if (r < eps) {
            st->done = 1;
            st->iterations = step;
        } else if (step == last_step) {
            st->iterations = step + 1;
        }
    }
}

} // namespace fracenc
