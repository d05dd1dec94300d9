// fracenc_kernels.hip — HIP/CDNA4 (gfx950) kernels of the range×domain search.
//
// Pipeline per frame:
//   pool_build      domain → decimated 2×2-sum vector D4 (n² u16, packed pairs) + −ΣD4²
//   search_valu     per (range, transform group, domain slice): exact integer error of every
//                   candidate with v_dot2_u32_u16 (range copies in VGPRs, domain vector
//                   broadcast from SGPRs), u64 atomicMin of the selection key per range
//   fit_winner      per range: re-derive the transform of the winning domain, the reference's
//                   least-squares contrast/brightness (FP64) and its fp32 error
//   fallback_grid   ranges whose best error leaves the exact fp32 regime: sequential fp32
//                   emulation of image/metrics.h over all candidates
#pragma once
#include "fracenc_common.h"

namespace fracenc {

__device__ inline int wave_sum_i(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    return v;
}

__device__ inline long long wave_sum_ll(long long v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    return v;
}

// ---------------------------------------------------------------------------
// pool_build: D4[i][j] is the 2×2 sum at domain pixel (2j, 2i): SamplerBilinear::sample's integer sum
// (image/sampler.h:21-38) for the identity transform at range pixel (j, i).  n ≥ 4: one lane per D4 row
// (n lanes per pool position p, bucket order): the row's two plane rows read as 32-bit words when the
// domain origin and the stride are 4-byte aligned (the ratio-2 grids at offset n ≥ 4 are), two cells per
// word pair — (w & 0x00ff00ff) + ((w >> 8) & 0x00ff00ff) over both rows is the packed u16 pair the pool
// stores; byte loads otherwise.  n = 2: one lane per pool word.  (One lane per pool word with 8 byte loads
// each ran the C4 quadtree's 261k-domain n = 4 level at 16 µs.)
// ---------------------------------------------------------------------------
__device__ inline uint32_t pair_sums(uint32_t w0, uint32_t w1)
{
    constexpr uint32_t M = 0x00ff00ffu;
    return (w0 & M) + ((w0 >> 8) & M) + (w1 & M) + ((w1 >> 8) & M);
}

template <int N>
__host__ __device__ constexpr int pool_lanes()
{
    return N >= 4 ? N : N * N / 2; // lanes per pool position
}

template <int N>
__global__ void __launch_bounds__(256) pool_build(const uint8_t* __restrict__ src, uint32_t sstride,
                                                  const frac_grid_item* __restrict__ doms,
                                                  const uint32_t* __restrict__ porig, uint32_t P,
                                                  uint32_t* __restrict__ pool, int32_t* __restrict__ negsd2)
{
    constexpr int NN = N * N, K2 = NN / 2, LPD = pool_lanes<N>();
    static_assert(64 % LPD == 0, "a pool position's lanes sit in one wave");
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t p = gid / LPD;
    const int k0 = (int)(gid % LPD);
    int sq = 0;
    if (p < P) {
        const frac_grid_item d = doms[porig[p]];
        if constexpr (N >= 4) {
            // lane k0: D4 row k0 = plane rows d.y + 2k0, + 1, columns d.x … d.x + 2N − 1; words N/2
            const uint8_t* r0 = src + (size_t)(d.y + 2u * (uint32_t)k0) * sstride + d.x;
            const uint8_t* r1 = r0 + sstride;
            uint32_t* out = pool + (size_t)p * K2 + (size_t)k0 * (N / 2);
            if ((((uintptr_t)r0 | sstride) & 3u) == 0) {
#pragma unroll
                for (int w = 0; w < N / 2; ++w) {
                    const uint32_t v = pair_sums(reinterpret_cast<const uint32_t*>(r0)[w],
                                                 reinterpret_cast<const uint32_t*>(r1)[w]);
                    const int lo = (int)(v & 0xffffu), hi = (int)(v >> 16);
                    sq += lo * lo + hi * hi;
                    out[w] = v;
                }
            } else {
#pragma unroll
                for (int w = 0; w < N / 2; ++w) {
                    const uint8_t* a = r0 + 4 * w;
                    const uint8_t* b = r1 + 4 * w;
                    const int lo = (int)a[0] + a[1] + b[0] + b[1], hi = (int)a[2] + a[3] + b[2] + b[3];
                    sq += lo * lo + hi * hi;
                    out[w] = (uint32_t)lo | ((uint32_t)hi << 16);
                }
            }
        } else {
            for (int k = k0; k < K2; k += LPD) {
                int v[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int qi = 2 * k + e;
                    const uint32_t x = d.x + 2u * (qi % N), y = d.y + 2u * (qi / N);
                    const uint8_t* r0 = src + (size_t)y * sstride + x;
                    v[e] = (int)r0[0] + (int)r0[1] + (int)r0[sstride] + (int)r0[sstride + 1];
                    sq += v[e] * v[e];
                }
                pool[(size_t)p * K2 + k] = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
            }
        }
    }
#pragma unroll
    for (int o = LPD / 2; o > 0; o >>= 1)
        sq += __shfl_xor(sq, o, 64);
    if (p < P && k0 == 0)
        negsd2[p] = -sq;
}

// ---------------------------------------------------------------------------
// search_valu<N, G, HITS>
//
// One wave = 64 ranges (one per lane, same classifier bucket) × one transform group
// (G transforms) × one slice [p_begin, p_end) of the bucket's domain pool.
// Lane state: G inverse-permuted copies of its range as packed u16 pairs (G·n²/2
// VGPRs), so that X_t = Σ_q copy_t[q]·D4[q] is one dot product against the
// UNPERMUTED domain vector, which is wave-uniform and therefore lives in SGPRs
// (s_load_dwordx16) and feeds v_dot2_u32_u16's scalar operand.
// Per candidate: w = 8·X − ΣD4² = C_r − S16 with C_r = 16Σr² (exact int32);
// the max over the group's transforms is kept per lane with strict '>' across
// domains (earliest domain wins ties), hits (S16 <= H) saturate to INT_MAX.
// ---------------------------------------------------------------------------
// Packs range pixels i0, i1 (bytes of the packed pixel dwords) as the u16 pair
// (i0 | i1 << 16) with one v_perm_b32: selectors 4..7 pick bytes of src0,
// 0..3 bytes of src1, 0x0c yields zero.
template <int N>
__device__ inline uint32_t pix_pair(const uint32_t (&pk)[(N * N + 3) / 4], int i0, int i1)
{
    const uint32_t sel = (uint32_t)(4 + (i0 & 3)) | (0x0cu << 8) | ((uint32_t)(i1 & 3) << 16) | (0x0cu << 24);
    return __builtin_amdgcn_perm(pk[i0 >> 2], pk[i1 >> 2], sel);
}

// Loads an N×N u8 block, four pixels per dword in row-major order.  Rows are read
// as aligned dwords and realigned with v_alignbit_b32 (any x), which keeps only a
// few loads in flight per row; the device plane has a slack row, so reading up to
// 4 bytes past a row end stays in bounds.
template <int N>
__device__ inline void load_range_packed(const uint8_t* __restrict__ plane, uint32_t stride, uint32_t x, uint32_t y,
                                         uint32_t (&pk)[(N * N + 3) / 4])
{
    if constexpr (N < 4) {
        uint32_t w = 0;
#pragma unroll
        for (int q = 0; q < N * N; ++q)
            w |= (uint32_t)plane[(size_t)(y + q / N) * stride + x + (q % N)] << (8 * q);
        pk[0] = w;
    } else {
        constexpr int W = N / 4; // dwords per row
#pragma unroll
        for (int r = 0; r < N; ++r) {
            const uintptr_t addr = (uintptr_t)(plane + (size_t)(y + r) * stride + x);
            const uint32_t* base = (const uint32_t*)(addr & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)(addr & 3);
            uint32_t w[W + 1];
#pragma unroll
            for (int i = 0; i <= W; ++i)
                w[i] = base[i];
#pragma unroll
            for (int i = 0; i < W; ++i)
                pk[r * W + i] = __builtin_amdgcn_alignbit(w[i + 1], w[i], sh * 8u); // shift in bits
        }
    }
}

template <int N, int G, int GROUP>
__device__ inline void build_copies(const uint32_t (&pk)[(N * N + 3) / 4], uint32_t (&cp)[G][N * N / 2])
{
#pragma unroll
    for (int j = 0; j < G; ++j) {
#pragma unroll
        for (int k = 0; k < N * N / 2; ++k) {
            const int t = GROUP * G + j;
            cp[j][k] = pix_pair<N>(pk, inv_index<N>(t, 2 * k), inv_index<N>(t, 2 * k + 1));
        }
    }
}

template <int N, int G, bool HITS>
__global__ void __launch_bounds__(256) search_valu(SearchArgs a)
{
    constexpr int NN = N * N, K2 = NN / 2;
    constexpr int KC = K2 < 32 ? K2 : 32; // dwords of the domain vector held in SGPRs at once
    const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wid >= a.nwork)
        return;
    const uint4 wk = a.work[wid];
    const uint32_t lane = threadIdx.x & 63u;
    const int ri = a.slot_range[wk.x + lane];
    const bool live = ri >= 0;
    const frac_grid_item rg = a.ranges[live ? ri : a.slot_range[wk.x]];

    // range pixels, four per dword (keeps the copy-building phase inside the
    // register budget of the main loop)
    uint32_t pix[(NN + 3) / 4];
    load_range_packed<N>(a.tgt, a.tstride, rg.x, rg.y, pix);
    int sum2 = 0;
#pragma unroll
    for (int q = 0; q < NN; ++q) {
        const int v = (int)((pix[q >> 2] >> (8 * (q & 3))) & 0xffu);
        sum2 += v * v;
    }
    const int Cr = 16 * sum2; // 16Σr² ≤ 2^28 for n ≤ 16
    const int hitlevel = Cr - a.hitH;

    uint32_t cp[G][K2];
    switch (wk.w) {
    case 0: build_copies<N, G, 0>(pix, cp); break;
    case 1: build_copies<N, G, 1>(pix, cp); break;
    case 2: if constexpr (G <= 2) build_copies<N, G, 2>(pix, cp); break;
    case 3: if constexpr (G <= 2) build_copies<N, G, 3>(pix, cp); break;
    case 4: if constexpr (G == 1) build_copies<N, G, 4>(pix, cp); break;
    case 5: if constexpr (G == 1) build_copies<N, G, 5>(pix, cp); break;
    case 6: if constexpr (G == 1) build_copies<N, G, 6>(pix, cp); break;
    default: if constexpr (G == 1) build_copies<N, G, 7>(pix, cp); break;
    }

    int best = INT_MIN;
    uint32_t bestp = 0;
    const uint32_t pe = wk.z;
    for (uint32_t p = wk.y; p < pe; ++p) {
        const uint32_t* __restrict__ dp = a.pool + (size_t)p * K2;
        uint32_t acc[G];
#pragma unroll
        for (int j = 0; j < G; ++j)
            acc[j] = 0;
#pragma unroll
        for (int kc = 0; kc < K2; kc += KC) {
            uint32_t dv[KC];
#pragma unroll
            for (int k = 0; k < KC; ++k)
                dv[k] = dp[kc + k];
#pragma unroll
            for (int j = 0; j < G; ++j)
#pragma unroll
                for (int k = 0; k < KC; ++k)
                    acc[j] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, dv[k]),
                                                    __builtin_bit_cast(ushort2_t, cp[j][kc + k]), acc[j], false);
        }
        const int ns = a.negsd2[p];
        int m = INT_MIN;
#pragma unroll
        for (int j = 0; j < G; ++j)
            m = max(m, (int)((acc[j] << 3) + (uint32_t)ns));
        if constexpr (HITS)
            m = m >= hitlevel ? INT_MAX : m;
        if (m > best) {
            best = m;
            bestp = p;
        }
        if constexpr (HITS) {
            if (__all(best == INT_MAX))
                break;
        }
    }
    if (live && best != INT_MIN) {
        unsigned long long key;
        if (HITS && best == INT_MAX)
            key = key_hit(bestp, 0);
        else
            key = key_miss((uint32_t)(Cr - best), bestp, 0);
        atomicMin(&a.best_key[ri], key);
    }
}

// ---------------------------------------------------------------------------
// fit_winner<N>: one lane group per range (fit_lanes: 16 lanes × 4 pixels at n = 8).
// Re-derives the winner's transform from the integer errors of its domain, then TransformMatcher::match_generic's fit
// (encode/transformmatcher.h:89-108).  All of ΣA, ΣA², ΣB = ΣD4/4, ΣAB = X/4
// are exact in FP64, so s is bit-exact in any summation order; o uses the
// reference's FMA-contracted form.  Distance = (S16/16)/(domain area), the
// reference's fp32 sum (exact here) divided in FP64 (image/metrics.h:49).
// ---------------------------------------------------------------------------
struct FitArgs {
    const uint8_t* tgt;
    uint32_t tstride;
    const frac_grid_item* ranges;
    const frac_grid_item* doms;
    const uint32_t* porig;
    const uint32_t* pool;
    const unsigned long long* best_key;
    uint32_t nr;
    uint32_t T;
    int64_t hitH;
    double smax;
    int all_fallback;
    frac_encode_item* out;
    RangeAux* aux;
    uint32_t* fb_count;
    uint32_t* fb_list;
    const DevPlan* plan = nullptr; // device-planned search: nr from the plan (the grid is a bound)
    // frac_set_tuple_sink: the fused resolvers (and fallback_grid) also write each range's 32-byte tuple here —
    // device memory or the caller's pinned host buffer, so the tuples cross PCIe while the resolve runs
    frac_tuple* tuples = nullptr;
};

// tp (a tuple sink): the same record as the (domain index, transform, s, o, rms) tuple
__device__ inline void write_fit(frac_encode_item& o, const frac_grid_item& rg, const frac_grid_item& d, int t,
                                 double sumA, double sumA2, double sumB, double sumAB, double N, double smax,
                                 double dist, frac_tuple* tp = nullptr, uint32_t dom = 0)
{
    const double tmp = (N * sumA2 - (sumA - 1) * sumA);
    double s = fabs(tmp) < 0.00001 ? 0.0 : (N * sumAB - sumA * sumB) / tmp;
    if (smax > 0.0)
        s = s > smax ? smax : (s < -smax ? -smax : s);
    const double br = __fma_rn(-s, sumA, sumB) / N;
    o.x = rg.x;
    o.y = rg.y;
    o.w = rg.w;
    o.h = rg.h;
    o.match.score.distance = dist;
    o.match.score.contrast = s;
    o.match.score.brightness = br;
    o.match.score.transform = t;
    o.match.score._pad = 0;
    o.match.x = d.x;
    o.match.y = d.y;
    o.match.sw = d.w;
    o.match.sh = d.h;
    if (tp) {
        frac_tuple u;
        u.domain = dom;
        u.transform = t;
        u.contrast = s;
        u.brightness = br;
        u.distance = dist;
        *tp = u;
    }
}

__device__ inline void write_default(frac_encode_item& o, const frac_grid_item& rg, frac_tuple* tp = nullptr)
{
    // item_match_t{} defaults (encode/datatypes.h:8-19): distance 1e5, s = o = 0, Id, (0,0), size (0,0)
    o.x = rg.x;
    o.y = rg.y;
    o.w = rg.w;
    o.h = rg.h;
    o.match.score.distance = 100000.0;
    o.match.score.contrast = 0.0;
    o.match.score.brightness = 0.0;
    o.match.score.transform = 0;
    o.match.score._pad = 0;
    o.match.x = 0;
    o.match.y = 0;
    o.match.sw = 0;
    o.match.sh = 0;
    if (tp) {
        frac_tuple u;
        u.domain = FRAC_NO_DOMAIN;
        u.transform = 0;
        u.contrast = 0.0;
        u.brightness = 0.0;
        u.distance = 100000.0;
        *tp = u;
    }
}

// lane groups of L: ranges per wave = 64 / L, 4 pixels per lane (n = 2: one lane per range)
template <int N>
constexpr int fit_lanes()
{
    return N * N >= 256 ? 64 : (N * N / 4 > 0 ? N * N / 4 : 1);
}

template <int L>
__device__ inline int group_sum_i(int v)
{
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    return v;
}

template <int N>
__device__ inline void fit_range(const FitArgs& a, uint32_t r, int sub)
{
    constexpr int NN = N * N, L = fit_lanes<N>(), PPL = NN / L;
    // whole lane groups leave together below, so the group sums only read live lanes
    if (r >= a.nr)
        return;
    const frac_grid_item rg = a.ranges[r];
    const unsigned long long key = a.best_key[r];
    if (key == kKeyNone) {
        if (sub == 0) {
            write_default(a.out[r], rg);
            a.aux[r] = RangeAux{0u, (uint32_t)kAuxEmpty};
        }
        return;
    }
    const uint32_t p = key_pos(key);
    // a miss-format key whose error meets H is a hit too (engines skip the hit sentinel
    // when H = 0, where a hit is the minimum error S16 = 0)
    const bool hit = (key >> 63) == 0 || (a.hitH >= 0 && (int64_t)((key >> 27) & 0xffffffffull) <= a.hitH);
    const frac_grid_item d = a.doms[a.porig[p]];
    const uint32_t* dp = a.pool + (size_t)p * (NN / 2);

    // every sum fits int32 for n ≤ 16 (ΣD4² ≤ 256·1020² < 2^31, X ≤ 256·255·1020 < 2^27)
    int sA = 0, sA2 = 0, sD = 0, sD2 = 0;
    int X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int q = sub * PPL + k;
        const int rv = a.tgt[(size_t)(rg.y + q / N) * a.tstride + rg.x + (q % N)];
        const uint32_t dw = dp[q >> 1];
        const int dv = (q & 1) ? (int)(dw >> 16) : (int)(dw & 0xffffu);
        sA += rv;
        sA2 += rv * rv;
        sD += dv;
        sD2 += dv * dv;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (t < (int)a.T) {
                // range pixel q meets D4[fwd(t, q)]
                const int f = fwd_index<N>(t, q);
                const uint32_t fw = dp[f >> 1];
                const int fv = (f & 1) ? (int)(fw >> 16) : (int)(fw & 0xffffu);
                X[t] += rv * fv;
            }
        }
    }
    sA = group_sum_i<L>(sA);
    sA2 = group_sum_i<L>(sA2);
    sD = group_sum_i<L>(sD);
    sD2 = group_sum_i<L>(sD2);
#pragma unroll
    for (int t = 0; t < 8; ++t)
        if (t < (int)a.T) // wave-uniform
            X[t] = group_sum_i<L>(X[t]);
    if (sub != 0)
        return;
    long long S16[8];
    long long minS = LLONG_MAX;
    int tsel = -1;
    for (int t = 0; t < (int)a.T; ++t) {
        S16[t] = 16 * (long long)sA2 - 8 * (long long)X[t] + sD2;
        if (S16[t] < minS)
            minS = S16[t];
    }
    if (hit) {
        for (int t = 0; t < (int)a.T; ++t)
            if (S16[t] <= a.hitH) {
                tsel = t;
                break;
            }
    } else {
        for (int t = 0; t < (int)a.T; ++t)
            if (S16[t] == minS)
                tsel = t; // later transform wins ties (transformmatcher.h:57,67 use <=)
    }
    uint32_t flags = hit ? (uint32_t)kAuxHit : 0u;
    if (a.all_fallback || (!hit && minS >= kExactLimit)) {
        flags |= kAuxFallback;
        const uint32_t idx = atomicAdd(a.fb_count, 1u);
        a.fb_list[idx] = r;
    }
    const double Nd = (double)NN;
    const double area = (double)(d.w * d.h);
    const double dist = ((double)S16[tsel] * 0.0625) / area;
    write_fit(a.out[r], rg, d, tsel, (double)sA, (double)sA2, (double)sD * 0.25, (double)X[tsel] * 0.25, Nd, a.smax,
              dist);
    a.aux[r] = RangeAux{p, flags};
}

// fit_rstat<N>: the fit for the Fourier path, whose resolve_dft recorded the winner's X_t,
// ΣD4, ΣD4², Σr and Σr² (MfmaResolveArgs::rstat): one thread per range, no pixel or pool
// reads; the transform comes from the selection key (resolve_dft emits hit-format keys for
// every hit, so a miss-format key is a miss). Same formulas and fallback rule as fit_winner.
//
// One range's record from its selection key and the winner's sums st = {X_t, ΣD4 | Σr << 16, ΣD4²,
// Σr²}: fit_rstat's body, also run by resolve_dft's wave when the fit is fused into it
// One range's record from its selection key and the winner's exact sums (X_t, ΣD4, Σr, ΣD4², Σr²):
// the resolve kernels' fused fit (resolve_dft through fit_rstat_range, resolve_mfma directly)
template <int N>
__device__ inline void fit_sums_range(const FitArgs& a, uint32_t r, unsigned long long key, long long X, long long sD,
                                      long long sA, long long sD2, long long sA2)
{
    constexpr int NN = N * N;
    const frac_grid_item rg = a.ranges[r];
    frac_tuple* tp = a.tuples ? a.tuples + r : nullptr;
    if (key == kKeyNone) {
        write_default(a.out[r], rg, tp);
        a.aux[r] = RangeAux{0u, (uint32_t)kAuxEmpty};
        return;
    }
    const uint32_t p = key_pos(key);
    // a miss-format key whose error meets H is a hit too (the resolve emits hit-format keys for hits)
    const bool hit = (key >> 63) == 0;
    const long long err = hit ? 0 : (long long)((key >> 27) & 0xfffffffffull);
    const int t = hit ? (int)(key & 7u) : (int)(a.T - 1 - (uint32_t)(key & 7u));
    if (!hit && err >= kExactLimit) { // fp32 regime: listed; fallback_grid writes the record
        a.aux[r] = RangeAux{p, (uint32_t)kAuxFallback};
        a.fb_list[atomicAdd(a.fb_count, 1u)] = r;
        return;
    }
    const uint32_t dom = a.porig[p];
    const frac_grid_item d = a.doms[dom];
    const long long S16 = 16 * sA2 - 8 * X + sD2;
    const double dist = ((double)S16 * 0.0625) / (double)(d.w * d.h);
    write_fit(a.out[r], rg, d, t, (double)sA, (double)sA2, (double)sD * 0.25, (double)X * 0.25, (double)NN, a.smax,
              dist, tp, dom);
    a.aux[r] = RangeAux{p, hit ? (uint32_t)kAuxHit : 0u};
}

// rgp / dp: the range's and the winner domain's items when the caller already holds them (resolve_dft),
// else loaded here
template <int N>
__device__ inline void fit_rstat_range(const FitArgs& a, uint32_t r, unsigned long long key, const uint4& st,
                                       const frac_grid_item* rgp = nullptr, const frac_grid_item* dp = nullptr)
{
    constexpr int NN = N * N;
    const frac_grid_item rg = rgp ? *rgp : a.ranges[r];
    frac_tuple* tp = a.tuples ? a.tuples + r : nullptr;
    if (key == kKeyNone) {
        write_default(a.out[r], rg, tp);
        a.aux[r] = RangeAux{0u, (uint32_t)kAuxEmpty};
        return;
    }
    const uint32_t p = key_pos(key);
    const bool hit = (key >> 63) == 0;
    const long long err = hit ? 0 : (long long)((key >> 27) & 0xffffffffull);
    const int t = hit ? (int)(key & 7u) : (int)(a.T - 1 - (uint32_t)(key & 7u));
    if (!hit && err >= kExactLimit) { // fp32 regime: listed; fallback_grid writes the record
        a.aux[r] = RangeAux{p, (uint32_t)kAuxFallback};
        a.fb_list[atomicAdd(a.fb_count, 1u)] = r;
        return;
    }
    const uint32_t dom = (!dp || tp) ? a.porig[p] : 0u; // the domain index (a tuple's, or to load the item)
    const frac_grid_item d = dp ? *dp : a.doms[dom];
    const long long X = st.x, sD = st.y & 0xffffu, sA = st.y >> 16, sD2 = st.z, sA2 = st.w;
    const long long S16 = 16 * sA2 - 8 * X + sD2;
    const double dist = ((double)S16 * 0.0625) / (double)(d.w * d.h);
    write_fit(a.out[r], rg, d, t, (double)sA, (double)sA2, (double)sD * 0.25, (double)X * 0.25, (double)NN, a.smax,
              dist, tp, dom);
    a.aux[r] = RangeAux{p, hit ? (uint32_t)kAuxHit : 0u};
}

template <int N>
__global__ void __launch_bounds__(256) fit_rstat(FitArgs a, const uint4* __restrict__ rstat)
{
    if (a.plan)
        a.nr = a.plan->nr;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.nr)
        return;
    const unsigned long long key = a.best_key[r];
    fit_rstat_range<N>(a, r, key, key == kKeyNone ? make_uint4(0u, 0u, 0u, 0u) : rstat[r]);
}

// one wave per 64 / L ranges (a grid-stride form over fewer waves measured slower)

template <int N>
__global__ void __launch_bounds__(256) fit_winner(FitArgs a)
{
    constexpr int L = fit_lanes<N>(), RPW = 64 / L;
    if (a.plan)
        a.nr = a.plan->nr;
    const int lane = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    fit_range<N>(a, w * RPW + (uint32_t)(lane / L), lane % L);
}

// ---------------------------------------------------------------------------
// The fp32 fallback (fallback_grid below): every candidate of a listed range's bucket with the reference's exact
// arithmetic: fp32 sum over range pixels in row-major order of
// (float(r) − float(2×2 sum)/4)² (image/metrics.h:37-50).  Selection key:
//   hit  (dist <= thr): (pos_local << 3) | t
//   miss:               (1 << 63) | (F_bits << 27) | (pos_local << 3) | (T−1−t)
// ---------------------------------------------------------------------------
struct FallbackArgs {
    const uint8_t* tgt;
    uint32_t tstride;
    const frac_grid_item* ranges;
    const frac_grid_item* doms;
    const uint32_t* porig;
    const uint32_t* pool;
    const uint2* rbucket; // per range: pool slice [x, y)
    const uint32_t* fb_count;
    const uint32_t* fb_list;
    uint32_t T;
    double thr;
    double smax;
    frac_encode_item* out;
    RangeAux* aux;
    frac_tuple* tuples = nullptr; // the run's tuple sink when its resolvers write one (FitArgs::tuples)
    // fallback_grid: per listed range the least key so far and its jobs done (kKeyNone / 0 between runs), and
    // the jobs per range (the domain chunks of the largest bucket)
    unsigned long long* fb_key = nullptr;
    uint32_t* fb_done = nullptr;
    uint32_t chunks = 0;
};

// one block per CU: an empty list (the usual case) costs the dispatch of these blocks only
constexpr unsigned kFallbackBlocks = 256;
constexpr uint32_t kFbChunk = 256; // fallback_grid: bucket domains per job (one per thread, every transform)

// one candidate (pool position bk.x + pl, transform t) of a range in the reference's fp32 arithmetic
// (rpix: the range's pixels as floats), as its selection key
template <int N>
__device__ inline unsigned long long fallback_key(const uint32_t* __restrict__ pool, const float* rpix, uint32_t p,
                                                  uint32_t pl, int t, uint32_t T, double thr)
{
    constexpr int NN = N * N;
    const uint32_t* dp = pool + (size_t)p * (NN / 2);
    float F = 0.0f;
    for (int q = 0; q < NN; ++q) {
        const int f = fwd_index<N>(t, q);
        const uint32_t fw = dp[f >> 1];
        const float smp = (float)((f & 1) ? (fw >> 16) : (fw & 0xffffu)) / 4.0f;
        const float val = __fsub_rn(rpix[q], smp);
        F = __fadd_rn(F, __fmul_rn(val, val));
    }
    const double dist = (double)F / (double)(4 * NN);
    if (dist <= thr)
        return ((unsigned long long)pl << 3) | (unsigned long long)t;
    return kKeyMiss | ((unsigned long long)__float_as_uint(F) << 27) | ((unsigned long long)pl << 3) |
           (unsigned long long)(T - 1 - t);
}

// range r's record from its least fp32 key k (kKeyNone: no candidate)
template <int N>
__device__ inline void fallback_record(const uint32_t* __restrict__ pool, const frac_grid_item* doms,
                                       const uint32_t* porig, uint32_t T, double smax, frac_encode_item* out,
                                       RangeAux* aux, uint32_t r, const frac_grid_item& rg, const uint2& bk,
                                       unsigned long long k, const float* rpix, frac_tuple* tuples = nullptr)
{
    constexpr int NN = N * N;
    frac_tuple* tp = tuples ? tuples + r : nullptr;
    if (k == kKeyNone) {
        write_default(out[r], rg, tp);
        aux[r] = RangeAux{0u, (uint32_t)kAuxEmpty};
        return;
    }
    const bool hit = (k >> 63) == 0;
    const uint32_t pl = (uint32_t)((k >> 3) & 0xffffffu);
    const int t = hit ? (int)(k & 7u) : (int)(T - 1 - (uint32_t)(k & 7u));
    const uint32_t p = bk.x + pl;
    const uint32_t dom = porig[p];
    const frac_grid_item d = doms[dom];
    const uint32_t* dp = pool + (size_t)p * (NN / 2);
    long long sA = 0, sA2 = 0, sD = 0, X = 0;
    float Fh = 0.0f;
    for (int q = 0; q < NN; ++q) {
        const int rv = (int)rpix[q];
        const uint32_t dw = dp[q >> 1];
        const int dv = (q & 1) ? (int)(dw >> 16) : (int)(dw & 0xffffu);
        const int f = fwd_index<N>(t, q);
        const uint32_t fw = dp[f >> 1];
        const int fv = (f & 1) ? (int)(fw >> 16) : (int)(fw & 0xffffu);
        sA += rv;
        sA2 += rv * rv;
        sD += dv;
        X += (long long)rv * fv;
        const float val = __fsub_rn(rpix[q], (float)fv / 4.0f);
        Fh = __fadd_rn(Fh, __fmul_rn(val, val));
    }
    const double dist = (double)Fh / (double)(d.w * d.h);
    write_fit(out[r], rg, d, t, (double)sA, (double)sA2, (double)sD * 0.25, (double)X * 0.25, (double)NN, smax,
              dist, tp, dom);
    aux[r] = RangeAux{p, (uint32_t)(kAuxFallback | (hit ? kAuxHit : 0u))};
}

// The reference's fp32 error of one (domain row, transform TT) (image/metrics.h:37-50): the row in registers,
// the transform a compile-time permutation, the range's pixels from LDS; every term exact, the sum sequential
// with one rounding per addition (__fadd_rn), as the reference's loop.
template <int N, int TT>
__device__ inline float fp32_error_t(const uint32_t* __restrict__ dp, const float* rpix)
{
    constexpr int NN = N * N, W = (NN + 1) / 2;
    if constexpr (N > 8) { // n = 16: a 128-word row would not stay in registers; the cells load as used
        float F = 0.0f;
#pragma unroll 16
        for (int q = 0; q < NN; ++q) {
            const int f = fwd_index<N>(TT, q);
            const uint32_t fw = dp[f >> 1];
            const float smp = (float)((f & 1) ? (fw >> 16) : (fw & 0xffffu)) / 4.0f;
            const float val = __fsub_rn(rpix[q], smp);
            F = __fadd_rn(F, __fmul_rn(val, val));
        }
        return F;
    }
    uint32_t w[N > 8 ? 1 : W];
    if constexpr (N > 8) {
    } else if constexpr (W % 4 == 0) {
#pragma unroll
        for (int k = 0; k < W / 4; ++k) {
            const uint4 v = reinterpret_cast<const uint4*>(dp)[k];
            w[4 * k] = v.x;
            w[4 * k + 1] = v.y;
            w[4 * k + 2] = v.z;
            w[4 * k + 3] = v.w;
        }
    } else { // n = 2: a row of two words
#pragma unroll
        for (int k = 0; k < W; ++k)
            w[k] = dp[k];
    }
    float F = 0.0f;
#pragma unroll
    for (int q = 0; q < NN; ++q) {
        const int f = fwd_index<N>(TT, q);
        const uint32_t fw = w[f >> 1];
        const float smp = (float)((f & 1) ? (fw >> 16) : (fw & 0xffffu)) / 4.0f;
        const float val = __fsub_rn(rpix[q], smp);
        F = __fadd_rn(F, __fmul_rn(val, val));
    }
    return F;
}

template <int N>
__device__ inline float fp32_error(const uint32_t* __restrict__ dp, const float* rpix, int t)
{
    switch (t) {
    case 0: return fp32_error_t<N, 0>(dp, rpix);
    case 1: return fp32_error_t<N, 1>(dp, rpix);
    case 2: return fp32_error_t<N, 2>(dp, rpix);
    case 3: return fp32_error_t<N, 3>(dp, rpix);
    case 4: return fp32_error_t<N, 4>(dp, rpix);
    case 5: return fp32_error_t<N, 5>(dp, rpix);
    case 6: return fp32_error_t<N, 6>(dp, rpix);
    default: return fp32_error_t<N, 7>(dp, rpix);
    }
}

// fallback_grid<N>: every range on the list (the fused resolvers list their fp32-regime ranges — only for n ≥ 8:
// below, S16 ≤ n²·1020² < 2^24 — and the all-fallback regime of a threshold at or above 2^24 lists them all) evaluated by the whole grid — a job is (listed range, chunk of kFbChunk bucket domains), one
// domain per thread and every transform; a block minimum of the selection keys (fallback_key's) goes into the
// range's fb_key with a 64-bit atomicMin, and the job completing the range's count writes its record
// (fallback_record) and resets the pair.  One wave per range (the resolvers' former in-wave fallback) took
// 328 ms for one C3 range (1,044,484 candidates); here the list's work spreads over every CU.  An empty list
// (the usual case) costs the blocks' dispatch.
template <int N>
__global__ void __launch_bounds__(256) fallback_grid(FallbackArgs a)
{
    constexpr int NN = N * N;
    __shared__ float rpix[NN];
    __shared__ unsigned long long red[4];
    __shared__ uint32_t last;
    const uint32_t count = *a.fb_count;
    const uint64_t jobs = (uint64_t)count * a.chunks;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint64_t job = blockIdx.x; job < jobs; job += gridDim.x) {
        const uint32_t e = (uint32_t)(job / a.chunks), ch = (uint32_t)(job % a.chunks);
        const uint32_t r = a.fb_list[e];
        const frac_grid_item rg = a.ranges[r];
        const uint2 bk = a.rbucket[r];
        __syncthreads(); // the previous job's LDS reads are done
        for (int q = threadIdx.x; q < NN; q += blockDim.x)
            rpix[q] = (float)(int16_t)a.tgt[(size_t)(rg.y + q / N) * a.tstride + rg.x + (q % N)];
        __syncthreads();
        unsigned long long best = kKeyNone;
        const uint32_t p = bk.x + ch * kFbChunk + threadIdx.x;
        if (p < bk.y) {
            const uint32_t* dp = a.pool + (size_t)p * (NN / 2);
            for (uint32_t t = 0; t < a.T; ++t) {
                const float F = fp32_error<N>(dp, rpix, (int)t);
                const double dist = (double)F / (double)(4 * NN);
                const uint32_t pl = p - bk.x;
                const unsigned long long key =
                    dist <= a.thr ? (((unsigned long long)pl << 3) | (unsigned long long)t)
                                  : (kKeyMiss | ((unsigned long long)__float_as_uint(F) << 27) |
                                     ((unsigned long long)pl << 3) | (unsigned long long)(a.T - 1 - t));
                best = key < best ? key : best;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long ob = ((unsigned long long)(uint32_t)__shfl_xor((int)(uint32_t)(best >> 32), o, 64) << 32) |
                                          (uint32_t)__shfl_xor((int)(uint32_t)best, o, 64);
            best = ob < best ? ob : best;
        }
        if (lane == 0)
            red[wv] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long b = red[0];
            for (uint32_t w = 1; w < blockDim.x / 64; ++w)
                b = red[w] < b ? red[w] : b;
            if (b != kKeyNone)
                atomicMin(a.fb_key + e, b);
            __threadfence(); // the key lands before the count that may let another job read it
            last = atomicAdd(a.fb_done + e, 1u) + 1u == a.chunks ? 1u : 0u;
            __threadfence();
        }
        __syncthreads();
        if (last && threadIdx.x == 0) {
            const unsigned long long k = atomicMin(a.fb_key + e, kKeyNone); // the final key (kKeyNone changes nothing)
            fallback_record<N>(a.pool, a.doms, a.porig, a.T, a.smax, a.out, a.aux, r, rg, bk, k, rpix, a.tuples);
            a.fb_key[e] = kKeyNone; // clean for the next run's list
            a.fb_done[e] = 0u;
        }
    }
}

// the fused fits' exit to the fp32 regime: a miss whose exact error is at least kExactLimit
__device__ inline bool key_needs_fallback(unsigned long long key)
{
    return key != kKeyNone && (key >> 63) != 0 && (long long)((key >> 27) & 0xfffffffffull) >= kExactLimit;
}

// ---------------------------------------------------------------------------
// pack_tuples: 64-byte results → 32-byte (domain index, transform, s, o, rms) tuples for
// the multi-GPU gather.  One thread per range.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) pack_tuples(const frac_encode_item* __restrict__ out,
                                                   const RangeAux* __restrict__ aux,
                                                   const uint32_t* __restrict__ porig, uint32_t nr,
                                                   frac_tuple* __restrict__ dst)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nr)
        return;
    const frac_encode_item o = out[r];
    const RangeAux x = aux[r];
    frac_tuple t;
    t.domain = (x.flags & kAuxEmpty) ? FRAC_NO_DOMAIN : porig[x.pos];
    t.transform = o.match.score.transform;
    t.contrast = o.match.score.contrast;
    t.brightness = o.match.score.brightness;
    t.distance = o.match.score.distance;
    dst[r] = t;
}

} // namespace fracenc
