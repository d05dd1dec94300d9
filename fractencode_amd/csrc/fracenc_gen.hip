// fracenc_gen.hip — the sampled form: every geometry other than "domain = 2 × range with
// n ∈ {2, 4, 8, 16}" (the decimate-then-permute path of the engines).
//
// TransformMatcher::matchTransformType (encode/transformmatcher.h:70-78) sends 16×16 domains with
// 4×4 ranges — the CLI default, encode/encode_parameters.h:6-7 — to match_16to4 (:113-144) and
// every other pair to match_generic (:80-111); both score a candidate with RootMeanSquare's
// different-size branch (image/metrics.h:37-50), which samples the domain at
//   (x·⌊S/n⌋, y·⌊S/n⌋)                       (metrics.h:40-45)
// while the fit samples it at
//   ((x·S)/n, (y·S)/n)                       (transformmatcher.h:94-95; match_16to4: (4x, 4y))
// — the same points whenever n divides S (per axis: ranges nw × nh and domains Sw × Sh may be
// rectangles, as the reference's Size32u items allow, with the x and y ratios of metrics.h:40-41).
// A sample is SamplerBilinear's 2×2 sum under the
// transform (image/sampler.h:21-38, image/transform.h:96-109).  At ratio 2 the samples of every
// transform are one permutation of the domain's 2×2-decimation; at any other ratio each transform
// samples a different set of 2×2 blocks (at ratio 4 the flipped ones start at offset 2).
//
// So this form builds one pool row per (domain, transform) — "virtual rows" v = p·T + (T−1−t), p
// the domain's pool position — holding the metric samples M in range-pixel order, and runs the
// engines' exhaustive searches over the rows with the single identity transform: the error of a
// candidate is S16 = Σ(4r − M)² exactly as on the ratio-2 path, the least key (S16, v) is the least
// error with ties to the earliest domain and then to the later transform (the reference's order,
// encode/TransformEstimator2.hpp:34, transformmatcher.h:57,67), and gen_fit turns v back into
// (domain, transform), moves a hit to the first transform of its domain that meets the threshold,
// and fits with the fit-point samples.  Range sizes other than 2, 4, 8, 16 (any side up to 256) search
// with gen_search.  The fp32 fallback (gen_fallback) replays the reference's sequential fp32 sum.
#include "fracenc_common.h"

namespace fracenc {

struct GenArgs {
    const uint8_t* src;     // domain plane
    uint32_t sstride;
    const uint8_t* tgt;     // range plane
    uint32_t tstride;
    const frac_grid_item* doms;
    const frac_grid_item* ranges;
    const uint32_t* porig;  // pool position → domain index
    uint32_t nw, nh, Sw, Sh; // range width / height, domain width / height
    uint32_t T, K2;          // transforms, dwords per pool row
    uint32_t* pool;         // [P·T][K2] metric samples, packed u16 pairs (zero padded)
    int32_t* negsd2;        // [P·T] −ΣM²
    uint32_t nrows;         // P·T
};

// SamplerBilinear::sample<·, t>'s integer 2×2 sum at patch-local (lx, ly) of an Sw×Sh domain at (dx, dy):
// the edge clamp of sampler.h:32-35, then the four offsets of Transform::generateSampleOffsets
// (transform.h:96-109): T(lx, ly), T(lx+1, ly), T(lx, ly+1), T(lx+1, ly+1).  For a rectangle the
// rotations map parts of the patch outside it, as in the reference; prepare() checks that every such
// read stays inside the plane (the reference reads out of bounds otherwise).
__device__ inline int gen_sample(const uint8_t* __restrict__ img, uint32_t stride, uint32_t dx, uint32_t dy,
                                 uint32_t Sw, uint32_t Sh, int t, uint32_t lx, uint32_t ly)
{
    if (lx == Sw - 1)
        --lx;
    if (ly == Sh - 1)
        --ly;
    const Aff a = lut(t);
    const int px = (int)dx + a.a0 * (int)lx + a.a1 * (int)ly + a.a2 * (int)(Sw - 1) + a.a3 * (int)(Sh - 1);
    const int py = (int)dy + a.a4 * (int)lx + a.a5 * (int)ly + a.a6 * (int)(Sw - 1) + a.a7 * (int)(Sh - 1);
    const ptrdiff_t s = (ptrdiff_t)stride;
    const uint8_t* p = img + (ptrdiff_t)py * s + px;
    return (int)p[0] + (int)p[a.a4 * s + a.a0] + (int)p[a.a5 * s + a.a1] + (int)p[(a.a4 + a.a5) * s + a.a0 + a.a1];
}

// One thread per virtual row v = p·T + (T−1−t): the nw·nh metric samples of domain porig[p] under t at
// (x·⌊Sw/nw⌋, y·⌊Sh/nh⌋) (image/metrics.h:40-45), as the pool row the engines read, and −ΣM².
__global__ void __launch_bounds__(256) gen_pool_build(GenArgs a)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= a.nrows)
        return;
    const uint32_t p = v / a.T;
    const int t = (int)(a.T - 1 - v % a.T);
    const frac_grid_item d = a.doms[a.porig[p]];
    const uint32_t rw = a.Sw / a.nw, rh = a.Sh / a.nh, NN = a.nw * a.nh;
    uint32_t* row = a.pool + (size_t)v * a.K2;
    int sq = 0;
    uint32_t x = 0, y = 0;
    for (uint32_t k = 0; k < a.K2; ++k) {
        uint32_t w = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t q = 2 * k + h;
            if (q < NN) {
                const int m = gen_sample(a.src, a.sstride, d.x, d.y, a.Sw, a.Sh, t, x * rw, y * rh);
                sq += m * m;
                w |= (uint32_t)m << (16 * h);
                if (++x == a.nw) {
                    x = 0;
                    ++y;
                }
            }
        }
        row[k] = w;
    }
    a.negsd2[v] = -sq;
}

// S16 = Σ(4r − M)² of range r (its pixels) against virtual row v: the reference's fp32 error × 16,
// exact in integers (image/metrics.h:45-49 with sample = M/4).
__device__ inline uint64_t gen_s16(const GenArgs& a, const frac_grid_item& rg, uint32_t v)
{
    const uint32_t* row = a.pool + (size_t)v * a.K2;
    const uint32_t NN = a.nw * a.nh;
    uint64_t s = 0;
    uint32_t x = 0, y = 0;
    for (uint32_t q = 0; q < NN; ++q) {
        const uint32_t w = row[q >> 1];
        const int m = (q & 1) ? (int)(w >> 16) : (int)(w & 0xffffu);
        const int e = 4 * (int)a.tgt[(size_t)(rg.y + y) * a.tstride + rg.x + x] - m;
        s += (uint64_t)(e * e);
        if (++x == a.nw) {
            x = 0;
            ++y;
        }
    }
    return s;
}

// gen_search: exhaustive search for range sizes without a templated engine (n ∉ {2, 4, 8, 16}).
// One wave per range; the lanes stride over the virtual rows of the range's bucket, each computing
// S16 of a whole row against the range pixels held in LDS (as 4r).  Keys in the engines' virtual
// format: (S16, v) for a miss, v for a hit (S16 ≤ H), least key per range.
struct GenSearchArgs {
    GenArgs g;
    const uint2* rbucket; // per range: virtual rows [x, y)
    uint32_t nr;
    int64_t hitH;
    unsigned long long* best_key;
};

// Range sides up to 256 search exactly (match_generic takes any size, transformmatcher.h:80-111; the CLI any
// 2 ≤ target < source, main.cpp:99): the largest S16 of a 256×256 range, 65,536 · 1020², stays below
// 2^36, the key's error field (fracenc_common.h key_miss).  Larger ranges run every candidate through
// gen_fallback's fp32 replay of the reference (prepare() sets all_fallback).
constexpr uint32_t kGenMaxN = 256;
// gen_search holds the range in LDS (as 4r) in chunks of kGenChunk pixels per wave
constexpr uint32_t kGenChunk = 4096;

__global__ void __launch_bounds__(256) gen_search(GenSearchArgs a)
{
    __shared__ int16_t r4[4][kGenChunk];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t r = blockIdx.x * 4u + wv;
    if (r >= a.nr)
        return;
    const GenArgs& g = a.g;
    const frac_grid_item rg = g.ranges[r];
    const uint32_t NN = g.nw * g.nh;
    auto load_chunk = [&](uint32_t c0) {
        __builtin_amdgcn_wave_barrier(); // the previous chunk's reads are done (the wave runs in lockstep)
        for (uint32_t q = lane; q < kGenChunk && c0 + q < NN; q += 64) {
            const uint32_t qq = c0 + q;
            r4[wv][q] = (int16_t)(4 * (int)g.tgt[(size_t)(rg.y + qq / g.nw) * g.tstride + rg.x + qq % g.nw]);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    };
    const uint2 seg = a.rbucket[r];
    unsigned long long best = kKeyNone;
    const bool one_chunk = NN <= kGenChunk;
    if (one_chunk)
        load_chunk(0);
    // rows in groups of 64, one per lane; a range larger than one chunk streams its chunks per group
    for (uint32_t v0 = seg.x; v0 < seg.y; v0 += 64) {
        const uint32_t v = v0 + lane;
        const uint32_t* row = g.pool + (size_t)min(v, seg.y - 1) * g.K2;
        uint64_t s = 0;
        for (uint32_t c0 = 0; c0 < NN; c0 += kGenChunk) {
            if (!one_chunk)
                load_chunk(c0);
            const uint32_t ce = min(NN, c0 + kGenChunk);
            for (uint32_t q = c0; q < ce; q += 2) {
                const uint32_t w = row[q >> 1];
                const int e0 = (int)r4[wv][q - c0] - (int)(w & 0xffffu);
                s += (uint64_t)(e0 * e0);
                if (q + 1 < ce) {
                    const int e1 = (int)r4[wv][q + 1 - c0] - (int)(w >> 16);
                    s += (uint64_t)(e1 * e1);
                }
            }
        }
        if (v < seg.y) {
            const unsigned long long key =
                (a.hitH >= 0 && (int64_t)s <= a.hitH) ? key_hit(v, 0) : key_miss(s, v, 0);
            best = key < best ? key : best;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o, 64);
        best = other < best ? other : best;
    }
    if (lane == 0)
        a.best_key[r] = best;
}

// gen_fit: one thread per range.  Decodes the engines' virtual key (row v = p·T + (T−1−t)); a hit
// moves to the first transform of domain p whose error meets H (the chain's early exit,
// transformmatcher.h:55,65; the search found the first domain holding a hit); a miss at or beyond
// 2^24 goes to gen_fallback.  The fit is match_generic's (transformmatcher.h:89-108) with the
// samples at ((x·Sw)/nw, (y·Sh)/nh); every sum is an exact integer in FP64.
struct GenFitArgs {
    GenArgs g;
    const unsigned long long* best_key;
    uint32_t nr;
    int64_t hitH;
    double smax;
    int all_fallback;
    frac_encode_item* out;
    RangeAux* aux;
    uint32_t* fb_count;
    uint32_t* fb_list;
};

__device__ inline void gen_write_fit(const GenArgs& g, frac_encode_item& o, const frac_grid_item& rg,
                                     const frac_grid_item& d, int t, uint64_t s16, double smax)
{
    long long sA = 0, sA2 = 0, sB = 0, sAB = 0;
    for (uint32_t y = 0; y < g.nh; ++y)
        for (uint32_t x = 0; x < g.nw; ++x) {
            const long long rv = g.tgt[(size_t)(rg.y + y) * g.tstride + rg.x + x];
            const long long b =
                gen_sample(g.src, g.sstride, d.x, d.y, g.Sw, g.Sh, t, (x * g.Sw) / g.nw, (y * g.Sh) / g.nh);
            sA += rv;
            sA2 += rv * rv;
            sB += b;
            sAB += rv * b;
        }
    const double dist = ((double)s16 * 0.0625) / (double)(d.w * d.h);
    // ΣA is ImageStatistics2::sum's: u16 arithmetic for ranges up to 16 wide (image/ImageStatistics.hpp:12-17,
    // .cpp:14-51), which wraps for a tall rectangle (16×32: up to 130,560); squares never reach 2^16
    const double N = (double)(g.nw * g.nh), sumA = g.nw <= 16 ? (double)(uint16_t)sA : (double)sA,
                 sumA2 = (double)sA2;
    const double sumB = (double)sB * 0.25, sumAB = (double)sAB * 0.25;
    const double tmp = (N * sumA2 - (sumA - 1) * sumA);
    double s = fabs(tmp) < 0.00001 ? 0.0 : (N * sumAB - sumA * sumB) / tmp;
    if (smax > 0.0)
        s = s > smax ? smax : (s < -smax ? -smax : s);
    o.x = rg.x;
    o.y = rg.y;
    o.w = rg.w;
    o.h = rg.h;
    o.match.score.distance = dist;
    o.match.score.contrast = s;
    o.match.score.brightness = __fma_rn(-s, sumA, sumB) / N;
    o.match.score.transform = t;
    o.match.score._pad = 0;
    o.match.x = d.x;
    o.match.y = d.y;
    o.match.sw = d.w;
    o.match.sh = d.h;
}

__device__ inline void gen_write_default(frac_encode_item& o, const frac_grid_item& rg)
{
    o.x = rg.x;
    o.y = rg.y;
    o.w = rg.w;
    o.h = rg.h;
    o.match.score.distance = 100000.0;
    o.match.score.contrast = 0.0;
    o.match.score.brightness = 0.0;
    o.match.score.transform = 0;
    o.match.score._pad = 0;
    o.match.x = o.match.y = o.match.sw = o.match.sh = 0;
}

__global__ void __launch_bounds__(256) gen_fit(GenFitArgs a)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.nr)
        return;
    const GenArgs& g = a.g;
    const frac_grid_item rg = g.ranges[r];
    const unsigned long long key = a.best_key[r];
    if (key == kKeyNone) {
        gen_write_default(a.out[r], rg);
        a.aux[r] = RangeAux{0u, (uint32_t)kAuxEmpty};
        return;
    }
    const uint32_t v = key_pos(key), T = g.T;
    const uint32_t p = v / T;
    int t = (int)(T - 1 - v % T);
    uint64_t s16 = gen_s16(g, rg, v);
    const bool hit = (key >> 63) == 0 || (a.hitH >= 0 && (int64_t)s16 <= a.hitH);
    if (hit) {
        for (uint32_t tt = 0; tt < T; ++tt) {
            const uint64_t s = gen_s16(g, rg, p * T + (T - 1 - tt));
            if ((int64_t)s <= a.hitH) {
                t = (int)tt;
                s16 = s;
                break;
            }
        }
    }
    if (a.all_fallback || (!hit && s16 >= (uint64_t)kExactLimit)) {
        a.aux[r] = RangeAux{p, (uint32_t)kAuxFallback};
        a.fb_list[atomicAdd(a.fb_count, 1u)] = r;
        return;
    }
    gen_write_fit(g, a.out[r], rg, g.doms[g.porig[p]], t, s16, a.smax);
    a.aux[r] = RangeAux{p, hit ? (uint32_t)kAuxHit : 0u};
}

// gen_fallback: one block per flagged range (grid-stride over the list).  Every candidate of the
// range's bucket in the reference's arithmetic: fp32 sum over the range pixels in row-major order of
// (r − M/4)² (image/metrics.h:42-48), FP64 division by the domain area; first hit in (domain,
// transform) order, else least fp32 error with ties to the earliest domain, then the later transform.
struct GenFallbackArgs {
    GenArgs g;
    const uint2* rbucket; // per range: virtual rows [x, y)
    const uint32_t* fb_count;
    const uint32_t* fb_list;
    double thr;
    double smax;
    frac_encode_item* out;
    RangeAux* aux;
};

// the range's pixels as int16 in LDS (the fp32 value of each is exact): up to 128×128; a larger
// range reads them from the plane (a wave-uniform address per step)
constexpr uint32_t kGenFbLds = 128 * 128;

__global__ void __launch_bounds__(256) gen_fallback(GenFallbackArgs a)
{
    __shared__ int16_t rpx[kGenFbLds];
    __shared__ unsigned long long red[256];
    const GenArgs& g = a.g;
    const uint32_t NN = g.nw * g.nh, T = g.T;
    const bool in_lds = NN <= kGenFbLds;
    frac_grid_item rg{};
    auto rpix = [&](uint32_t q) -> float {
        return in_lds ? (float)rpx[q] : (float)(int16_t)g.tgt[(size_t)(rg.y + q / g.nw) * g.tstride + rg.x + q % g.nw];
    };
    const uint32_t count = *a.fb_count;
    for (uint32_t e = blockIdx.x; e < count; e += gridDim.x) {
        const uint32_t r = a.fb_list[e];
        rg = g.ranges[r];
        const uint2 seg = a.rbucket[r];
        const uint32_t p0 = seg.x / T; // the bucket's first pool position
        __syncthreads();
        for (uint32_t q = threadIdx.x; in_lds && q < NN; q += blockDim.x)
            rpx[q] = (int16_t)g.tgt[(size_t)(rg.y + q / g.nw) * g.tstride + rg.x + q % g.nw];
        __syncthreads();
        const double area = (double)(g.Sw * g.Sh);
        unsigned long long best = kKeyNone;
        for (uint32_t v = seg.x + threadIdx.x; v < seg.y; v += blockDim.x) {
            const uint32_t* row = g.pool + (size_t)v * g.K2;
            float F = 0.0f;
            for (uint32_t q = 0; q < NN; ++q) {
                const uint32_t w = row[q >> 1];
                const float smp = (float)((q & 1) ? (w >> 16) : (w & 0xffffu)) / 4.0f;
                const float val = __fsub_rn(rpix(q), smp);
                F = __fadd_rn(F, __fmul_rn(val, val));
            }
            const uint32_t pl = v / T - p0, tc = v % T; // tc = T − 1 − t
            const unsigned long long key =
                (double)F / area <= a.thr ? key_hit(pl, T - 1 - tc)
                                          : kKeyMiss | ((unsigned long long)__float_as_uint(F) << 27) |
                                                ((unsigned long long)pl << 3) | (unsigned long long)tc;
            best = key < best ? key : best;
        }
        red[threadIdx.x] = best;
        __syncthreads();
        for (uint32_t s = blockDim.x / 2; s > 0; s >>= 1) {
            if (threadIdx.x < s && red[threadIdx.x + s] < red[threadIdx.x])
                red[threadIdx.x] = red[threadIdx.x + s];
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            const unsigned long long k = red[0];
            if (k == kKeyNone) {
                gen_write_default(a.out[r], rg);
                a.aux[r] = RangeAux{0u, (uint32_t)kAuxEmpty};
            } else {
                const bool hit = (k >> 63) == 0;
                const uint32_t p = p0 + key_pos(k);
                const int t = hit ? (int)(k & 7u) : (int)(T - 1 - (uint32_t)(k & 7u));
                const frac_grid_item d = g.doms[g.porig[p]];
                // the winner's fp32 error, recomputed in order from its row
                const uint32_t* row = g.pool + (size_t)(p * T + (T - 1 - (uint32_t)t)) * g.K2;
                float F = 0.0f;
                for (uint32_t q = 0; q < NN; ++q) {
                    const uint32_t w = row[q >> 1];
                    const float smp = (float)((q & 1) ? (w >> 16) : (w & 0xffffu)) / 4.0f;
                    const float val = __fsub_rn(rpix(q), smp);
                    F = __fadd_rn(F, __fmul_rn(val, val));
                }
                gen_write_fit(g, a.out[r], rg, d, t, 0, a.smax);
                a.out[r].match.score.distance = (double)F / area;
                a.aux[r] = RangeAux{p, (uint32_t)(kAuxFallback | (hit ? kAuxHit : 0u))};
            }
        }
    }
}

} // namespace fracenc
