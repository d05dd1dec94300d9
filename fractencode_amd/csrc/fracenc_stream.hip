// fracenc_stream.hip — FRC1 quantized stream packed on the device.
//
//   frc1_minmax   per range: contrast / brightness into order-preserving u64 keys,
//                 workgroup reduce, one atomicMin / atomicMax per workgroup and field
//   frc1_records  per range: domain index on the lattice (index = n_domains when the range
//                 had no eligible domain), transform, Frac::Quantizer codes
//                 (encode/Quantizer.hpp:7-45: step = |max − min| / 2^bits,
//                 q = min(2^bits − 1, floor((v − min) / step)), FP64 as the reference),
//                 concatenated LSB-first into one u64 record
//   frc1_words    per 32-bit output word: the bits of the records it overlaps (records are
//                 `width` bits, word j holds stream bits [32j, 32j + 32))
// fractencode_amd/codec.py is the host restatement the tests compare against byte for byte.
#include "fracenc_common.h"

namespace fracenc {

// order-preserving map of an IEEE double to u64 (negative: all bits flipped; else sign set)
__host__ __device__ inline unsigned long long dkey(double v)
{
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
__host__ __device__ inline double dkey_inv(unsigned long long k)
{
    const unsigned long long b = (k >> 63) ? (k & ~(1ull << 63)) : ~k;
    return __builtin_bit_cast(double, b);
}

struct Frc1MinMax {
    unsigned long long cmin, cmax, bmin, bmax; // dkey()
};

__global__ void __launch_bounds__(256) frc1_minmax(const frac_encode_item* __restrict__ out, uint32_t n,
                                                   Frc1MinMax* __restrict__ mm)
{
    unsigned long long v[4] = {~0ull, 0ull, ~0ull, 0ull};
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        const unsigned long long c = dkey(out[r].match.score.contrast), b = dkey(out[r].match.score.brightness);
        v[0] = min(v[0], c);
        v[1] = max(v[1], c);
        v[2] = min(v[2], b);
        v[3] = max(v[3], b);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        v[0] = min(v[0], (unsigned long long)__shfl_xor(v[0], o, 64));
        v[1] = max(v[1], (unsigned long long)__shfl_xor(v[1], o, 64));
        v[2] = min(v[2], (unsigned long long)__shfl_xor(v[2], o, 64));
        v[3] = max(v[3], (unsigned long long)__shfl_xor(v[3], o, 64));
    }
    if ((threadIdx.x & 63u) == 0) {
        atomicMin(&mm->cmin, v[0]);
        atomicMax(&mm->cmax, v[1]);
        atomicMin(&mm->bmin, v[2]);
        atomicMax(&mm->bmax, v[3]);
    }
}

struct Frc1Args {
    const frac_encode_item* out;
    uint32_t n;
    uint32_t dstride, dcols, ndomains;
    uint32_t index_bits, t_bits, c_bits, b_bits;
    const Frc1MinMax* mm;
    unsigned long long* rec; // [n]
};

// Frac::Quantizer::quantized; a degenerate field (max == min) codes every value as 0
__device__ inline unsigned long long quantize(double v, double lo, double hi, uint32_t bits)
{
    if (!(hi > lo))
        return 0ull;
    const double step = fabs(hi - lo) / (double)(1u << bits);
    const double q = floor((v - lo) / step);
    const double qmax = (double)((1u << bits) - 1u);
    return (unsigned long long)(q < qmax ? q : qmax);
}

__global__ void __launch_bounds__(256) frc1_records(Frc1Args a)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.n)
        return;
    const frac_encode_item e = a.out[r];
    const bool has = e.match.sw != 0 && e.match.sh != 0;
    const unsigned long long idx =
        has ? (unsigned long long)(e.match.y / a.dstride) * a.dcols + e.match.x / a.dstride : a.ndomains;
    const double cmin = dkey_inv(a.mm->cmin), cmax = dkey_inv(a.mm->cmax);
    const double bmin = dkey_inv(a.mm->bmin), bmax = dkey_inv(a.mm->bmax);
    unsigned long long w = idx;
    uint32_t sh = a.index_bits;
    w |= (unsigned long long)(uint32_t)e.match.score.transform << sh;
    sh += a.t_bits;
    w |= quantize(e.match.score.contrast, cmin, cmax, a.c_bits) << sh;
    sh += a.c_bits;
    w |= quantize(e.match.score.brightness, bmin, bmax, a.b_bits) << sh;
    a.rec[r] = w;
}

__global__ void __launch_bounds__(256) frc1_words(const unsigned long long* __restrict__ rec, uint32_t n,
                                                  uint32_t width, uint64_t nwords, uint32_t* __restrict__ words)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nwords)
        return;
    const uint64_t b0 = 32 * j, b1 = b0 + 32, total = (uint64_t)n * width;
    uint32_t word = 0;
    for (uint64_t k = b0 / width; k < n && k * width < b1; ++k) {
        const uint64_t rb = k * width; // record k occupies [rb, rb + width)
        // the record's bits in this word: stream bits [lo, hi) ↔ record bits [lo − rb, hi − rb)
        const uint64_t lo = rb > b0 ? rb : b0;
        uint64_t hi = rb + width < b1 ? rb + width : b1;
        hi = hi < total ? hi : total;
        const uint32_t len = (uint32_t)(hi - lo); // 1..32
        const unsigned long long chunk = (rec[k] >> (lo - rb)) & (len == 64 ? ~0ull : ((1ull << len) - 1ull));
        word |= (uint32_t)(chunk << (lo - b0));
    }
    words[j] = word;
}

} // namespace fracenc
