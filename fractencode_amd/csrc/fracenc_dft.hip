// fracenc_dft.hip — rotation-group (C4) Fourier form of the MFMA search, n = 8, T = 4.
//
// The reference's four transforms (Id, R90, R180, R270; transformmatcher.h:41-45) act on
// the n×n decimated grid as g^t for the single permutation g = fwd(1): fwd(t) = g^t
// (checked at compile time below).  The 64 pixels split into 16 orbits {q, gq, g²q, g³q}
// and with a = r − 128 (range), b = D4 − 512 (domain), per orbit o, k = 0..3:
//
//   Z_t = Σ_p a(p)·b(g^t p) = Σ_o Σ_k a_{o,k}·b_{o,k+t}           (cyclic correlation)
//
// The length-4 DFT diagonalises it.  With per-orbit components
//   Â0 = Σa, Â2 = a0−a1+a2−a3, α = a0−a2, β = a1−a3   (range; B̂0, B̂2, γ, δ for the domain)
// and the four products  P0 = ΣÂ0B̂0,  P2 = ΣÂ2B̂2,  Pr = Σ(αγ+βδ),  Pi = Σ(βγ−αδ):
//
//   4Z_0 = A + 2Pr,  4Z_2 = A − 2Pr,  4Z_1 = B − 2Pi,  4Z_3 = B + 2Pi,   A = P0+P2, B = P0−P2
//
// so  max_t 4Z_t = max(A + 2|Pr|, B + 2|Pi|)  and the least error over the four transforms is
//
//   S16_min − 16Σa² = w = Σb² − 2·max_t 4Z_t          (S16 = Σ(4r − D4)² = 16Σa² − 8Z + Σb²)
//
// Cost per (32 domains × 32 ranges): 6 MFMA 32x32x16 (P0, P2: K=16; Pr, Pi: K=32) instead
// of T·n²/16 = 16, and 6.5 VALU per (range, domain) instead of 4 × 1.5.
//
// Exactness (f16 operands, f32 accumulate, all values integers):
//   operands  |Â0| ≤ 512, |Â2| ≤ 510, |α|,|β| ≤ 255;  |B̂0| ≤ 2048, |B̂2| ≤ 2040, |γ|,|δ| ≤ 1020
//             — integers of magnitude ≤ 2048 are exact in f16;
//   products  every partial sum of P0, P2 (16 terms ≤ 2^20) and Pr, Pi (32 terms ≤ 2^18)
//             is an integer of magnitude ≤ 2^24: exact in any accumulation order;
//   epilogue  A = 2Σ(s_a s_b + u_a u_b) (s = x0+x2, u = x1+x3) is an even integer, |A| ≤ 2^24,
//             likewise B; A ± 2Pr and B ± 2Pi are 4Z_t with |4Z_t| ≤ 4·64·128·512 = 2^24:
//             each op's exact result is representable, so every step is exact;
//             w = fma(m, −2, Σb²) is exact whenever |w| ≤ 2^24, which holds for every
//             candidate in the exact regime S16 < 2^24 (w = S16 − 16Σa², 16Σa² ≤ 2^24).
//   Candidates with S16 ≥ 2^24 may round, but rounding is monotone: w ≥ 2^24 − 16Σa² (an
//   exactly representable bound) stays ≥ it, so they never beat or tie an exact-regime
//   candidate, and a range whose minimum reaches that bound is sent to the fp32 fallback
//   (App. A.3), exactly as the direct engine does.
// The per-lane chunk minimum of w and the tile it appeared in feed resolve_dft, which
// re-derives the exact (domain, transform) inside the chunk with integer arithmetic.
#include "fracenc_common.h"

namespace fracenc {

template <int N>
struct Orbits4 {
    int p[N * N / 4][4]; // p[o][k] = g^k(q_o)
};

template <int N>
constexpr Orbits4<N> make_orbits4()
{
    Orbits4<N> r{};
    bool seen[N * N] = {};
    int o = 0;
    for (int q = 0; q < N * N; ++q) {
        if (seen[q])
            continue;
        int p = q;
        for (int k = 0; k < 4; ++k) {
            r.p[o][k] = p;
            seen[p] = true;
            p = fwd_index<N>(1, p);
        }
        ++o;
    }
    return r;
}

template <int N>
constexpr bool orbits4_valid()
{
    // fwd(t) = g^t for t = 0..3, g^4 = id, and every orbit has exactly four pixels
    for (int q = 0; q < N * N; ++q) {
        int p = q;
        for (int t = 0; t < 4; ++t) {
            if (fwd_index<N>(t, q) != p)
                return false;
            p = fwd_index<N>(1, p);
        }
        if (p != q)
            return false;
    }
    const Orbits4<N> r = make_orbits4<N>();
    int count[N * N] = {};
    for (int o = 0; o < N * N / 4; ++o)
        for (int k = 0; k < 4; ++k)
            ++count[r.p[o][k]];
    for (int q = 0; q < N * N; ++q)
        if (count[q] != 1)
            return false;
    return true;
}

static_assert(orbits4_valid<8>(), "the reference's rotations must be the powers of Rotate_90 with 4-orbits");
constexpr Orbits4<8> kOrb8 = make_orbits4<8>();
constexpr float kDftPadConst = 1.0e30f; // Σb² of padding rows: w ≈ 1e30 never wins

// ---------------------------------------------------------------------------
// dft_domain_prep: pool (u16 D4) → per 32-domain tile the A fragments of the four
// K-steps [B̂0 | B̂2 | γ | δ] (lane l: row l&31, orbit 8(l>>5) + j) and Σb² per row
// in the [2][16] lane-half layout of the epilogue.  One thread per (tile, row).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) dft_domain_prep(MfmaDomainPrepArgs a)
{
    constexpr int N = 8, NN = 64, NO = 16;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= a.ntiles * 32u)
        return;
    const uint32_t tile = gid >> 5, row = gid & 31u;
    const int p = a.tile_pos[gid];
    int b[NN];
    int sb2 = 0;
#pragma unroll
    for (int k = 0; k < NN / 2; ++k) {
        const uint32_t w = p >= 0 ? a.pool[(size_t)p * (NN / 2) + k] : 0x02000200u; // padding: b = 0
        b[2 * k] = (int)(w & 0xffffu) - 512;
        b[2 * k + 1] = (int)(w >> 16) - 512;
    }
#pragma unroll
    for (int k = 0; k < NN; ++k)
        sb2 += b[k] * b[k];
    _Float16 comp[4][NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) {
        const int b0 = b[kOrb8.p[o][0]], b1 = b[kOrb8.p[o][1]], b2 = b[kOrb8.p[o][2]], b3 = b[kOrb8.p[o][3]];
        comp[0][o] = (_Float16)(b0 + b1 + b2 + b3);
        comp[1][o] = (_Float16)(b0 - b1 + b2 - b3);
        comp[2][o] = (_Float16)(b0 - b2);
        comp[3][o] = (_Float16)(b1 - b3);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            _Float16 v8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                v8[j] = comp[s][8 * h + j];
            a.dtiles[((size_t)tile * 4 + s) * 64 + row + 32 * h] = __builtin_bit_cast(uint4, v8);
        }
    const float e = p >= 0 ? (float)sb2 : kDftPadConst; // Σb² ≤ 64·512² = 2^24: exact
    const uint32_t h = (row >> 2) & 1u, i = (row & 3u) + 4u * (row >> 3);
    a.dconst[(size_t)tile * 32 + h * 16 + i] = __float_as_uint(e);
    (void)N;
}

// ---------------------------------------------------------------------------
// dft_range_prep: per range block the six B fragments
//   f0 = Â0, f1 = Â2  (K=16 each),  Pr: [f2 = α | f3 = β],  Pi: [f4 = β | f5 = −α]
// (lane l: range slot l&31, orbit 8(l>>5) + j) and 16Σa² per slot.  One thread per slot.
// ---------------------------------------------------------------------------
constexpr int kDftRangeFrags = 6;

__global__ void __launch_bounds__(256) dft_range_prep(MfmaRangePrepArgs a)
{
    constexpr int N = 8, NN = 64, NO = 16;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= a.nblocks * 32u)
        return;
    const uint32_t b = gid >> 5, col = gid & 31u;
    const int ri = a.slot_range[gid];
    int av[NN];
    int sa2 = 0;
    if (ri >= 0) {
        const frac_grid_item rg = a.ranges[ri];
#pragma unroll
        for (int q = 0; q < NN; ++q) {
            av[q] = (int)a.tgt[(size_t)(rg.y + q / N) * a.tstride + rg.x + (q % N)] - 128;
            sa2 += av[q] * av[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < NN; ++q)
            av[q] = 0;
    }
    _Float16 comp[kDftRangeFrags][NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) {
        const int a0 = av[kOrb8.p[o][0]], a1 = av[kOrb8.p[o][1]], a2 = av[kOrb8.p[o][2]], a3 = av[kOrb8.p[o][3]];
        comp[0][o] = (_Float16)(a0 + a1 + a2 + a3);
        comp[1][o] = (_Float16)(a0 - a1 + a2 - a3);
        comp[2][o] = (_Float16)(a0 - a2);
        comp[3][o] = (_Float16)(a1 - a3);
        comp[4][o] = (_Float16)(a1 - a3);
        comp[5][o] = (_Float16)(a2 - a0);
    }
#pragma unroll
    for (int f = 0; f < kDftRangeFrags; ++f)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            _Float16 v8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                v8[j] = comp[f][8 * h + j];
            a.rfrags[((size_t)b * kDftRangeFrags + f) * 64 + col + 32 * h] = __builtin_bit_cast(uint4, v8);
        }
    a.rconst[gid] = ri >= 0 ? (uint32_t)(16 * sa2) : 0u; // 16Σa² ≤ 2^24
}

// ---------------------------------------------------------------------------
// search_dft<HITS>: the search_mfma work decomposition (workgroup = 4 waves = 4 range
// blocks of one bucket, domain tiles staged through LDS, 4 tiles per double-buffered
// stage); per lane the chunk minimum of w over its 16 rows × the stage's tiles and all
// four transforms.  Entries: [nwork*4][64] {float bits of min w (−inf = hit), tile}.
// ---------------------------------------------------------------------------
__device__ inline float dft_row(float p0, float p2, float pr, float pi, float sb2)
{
    const float A = p0 + p2, B = p0 - p2;
    const float x1 = __builtin_fmaf(__builtin_fabsf(pr), 2.0f, A); // max(4Z_0, 4Z_2)
    const float x2 = __builtin_fmaf(__builtin_fabsf(pi), 2.0f, B); // max(4Z_1, 4Z_3)
    return __builtin_fmaf(__builtin_fmaxf(x1, x2), -2.0f, sb2);    // min_t S16 − 16Σa²
}

template <int VAR>
__device__ inline float dft_tile_min(const half8_t (&af)[4], const half8_t (&bf)[kDftRangeFrags], const float (&e)[16],
                                     float m)
{
    const floatx16_t z = {};
    const floatx16_t p0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[0], z, 0, 0, 0);
    const floatx16_t p2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[1], z, 0, 0, 0);
    floatx16_t pr = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bf[2], z, 0, 0, 0);
    floatx16_t pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bf[4], z, 0, 0, 0);
    pr = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bf[3], pr, 0, 0, 0);
    pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bf[5], pi, 0, 0, 0);
    float m0 = m, m1 = __builtin_inff();
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
        m0 = __builtin_fminf(__builtin_fminf(m0, dft_row(p0[i], p2[i], pr[i], pi[i], e[i])),
                             dft_row(p0[i + 1], p2[i + 1], pr[i + 1], pi[i + 1], e[i + 1]));
        m1 = __builtin_fminf(__builtin_fminf(m1, dft_row(p0[i + 2], p2[i + 2], pr[i + 2], pi[i + 2], e[i + 2])),
                             dft_row(p0[i + 3], p2[i + 3], pr[i + 3], pi[i + 3], e[i + 3]));
    }
    (void)VAR;
    return __builtin_fminf(m0, m1);
}

template <int VAR>
__device__ inline float dft_compute_stage(const uint4* __restrict__ la, uint32_t nt, uint32_t lane,
                                          const half8_t (&bf)[kDftRangeFrags])
{
    const uint4* lc = la + nt * 4u * 64u;
    const uint32_t h = lane >> 5;
    float cm = __builtin_inff();
    for (uint32_t q = 0; q < nt; ++q) {
        half8_t af[4];
#pragma unroll
        for (int s = 0; s < 4; ++s)
            af[s] = __builtin_bit_cast(half8_t, la[(q * 4 + s) * 64 + lane]);
        float e[16];
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
            const uint4 v = lc[q * 8 + h * 4 + c4];
            e[4 * c4 + 0] = __uint_as_float(v.x);
            e[4 * c4 + 1] = __uint_as_float(v.y);
            e[4 * c4 + 2] = __uint_as_float(v.z);
            e[4 * c4 + 3] = __uint_as_float(v.w);
        }
        cm = dft_tile_min<VAR>(af, bf, e, cm);
    }
    return cm;
}

template <bool HITS, int VAR>
__global__ void __launch_bounds__(256) search_dft(MfmaSearchArgs a)
{
    constexpr int KS = 4;
    constexpr int STAGE = kTilesPerStage * KS * 64 + kTilesPerStage * 8;
    __shared__ uint4 lds0[STAGE];
    __shared__ uint4 lds1[STAGE];
    const uint4 wk = a.work[blockIdx.x];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const bool active = wv < wk.y;
    const uint32_t blk = wk.x + (active ? wv : 0u);

    half8_t bf[kDftRangeFrags];
#pragma unroll
    for (int f = 0; f < kDftRangeFrags; ++f)
        bf[f] = __builtin_bit_cast(half8_t, a.rfrags[((size_t)blk * kDftRangeFrags + f) * 64 + lane]);
    float hl = 0.0f;
    if constexpr (HITS) // S16 ≤ H  ⇔  w ≤ H − 16Σa²  (both exact integers below 2^24)
        hl = (float)((int32_t)a.hitH - (int32_t)a.rconst[blk * 32 + (lane & 31u)]);

    float best = __builtin_inff();
    uint32_t btile = 0;
    auto finish_stage = [&](float cm, uint32_t tb) {
        if constexpr (HITS)
            cm = cm <= hl ? -__builtin_inff() : cm; // any hit in the chunk: the first-hit chunk wins
        if (cm < best) {
            best = cm;
            btile = tb;
        }
    };
    const uint32_t nstage = (wk.w - wk.z + kTilesPerStage - 1) / kTilesPerStage;
    auto stage_nt = [&](uint32_t st) { return min((uint32_t)kTilesPerStage, wk.w - (wk.z + st * kTilesPerStage)); };
    if (nstage)
        stage_tiles<KS>(lds0, a.dtiles, a.dconst, wk.z, stage_nt(0));
    for (uint32_t st = 0; st < nstage; st += 2) {
        {
            const uint32_t tb = wk.z + st * kTilesPerStage;
            __syncthreads();
            if (st + 1 < nstage)
                stage_tiles<KS>(lds1, a.dtiles, a.dconst, tb + kTilesPerStage, stage_nt(st + 1));
            finish_stage(dft_compute_stage<VAR>(lds0, stage_nt(st), lane, bf), tb);
        }
        if (st + 1 < nstage) {
            const uint32_t tb = wk.z + (st + 1) * kTilesPerStage;
            __syncthreads();
            if (st + 2 < nstage)
                stage_tiles<KS>(lds0, a.dtiles, a.dconst, tb + kTilesPerStage, stage_nt(st + 2));
            finish_stage(dft_compute_stage<VAR>(lds1, stage_nt(st + 1), lane, bf), tb);
        }
    }
    if (active)
        a.entries[(size_t)(blockIdx.x * 4u + wv) * 64 + lane] = make_uint2(__float_as_uint(best), btile);
}

// ---------------------------------------------------------------------------
// resolve_dft: one wave per range (resolve_mfma's lane map: tile row i = l>>2, pixel
// slice g = l&3).  The least entry w over the block's splits and lane halves gives the
// target error S16 = w + 16Σa² (exact regime) or flags the range for the fp32 fallback;
// the chunk(s) holding it are re-evaluated with exact integers for all four transforms,
// keeping the least selection key (first hit in (domain, transform) order, else least
// error with ties to the earliest domain, then the later transform).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) resolve_dft(MfmaResolveArgs a)
{
    constexpr int N = 8, NN = 64, PG = 16, T = 4;
    const uint32_t r = blockIdx.x * 4u + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= a.nr)
        return;
    const uint32_t slot = a.range_slot[r];
    const uint32_t blk = slot >> 5, col = slot & 31u;
    const uint32_t e0 = a.blk_ptr[blk], e1 = a.blk_ptr[blk + 1];
    const uint32_t nent = (e1 - e0) * 2u;
    float vmin = __builtin_inff();
    for (uint32_t j = lane; j < nent; j += 64)
        vmin = __builtin_fminf(vmin, __uint_as_float(a.entries[(size_t)a.blk_ent[e0 + j / 2] * 64 + col + 32 * (j & 1)].x));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        vmin = __builtin_fminf(vmin, __shfl_xor(vmin, o, 64));
    if (!(vmin < 1.0e29f))
        return; // only padding rows: no eligible domain, best_key stays "none"
    const int64_t sa16 = (int64_t)a.rconst[slot];
    const bool exact = vmin < (float)(kExactLimit - sa16);
    const int64_t target = exact && vmin != -__builtin_inff() ? (int64_t)vmin + sa16 : -1;
    const bool hit = a.hitH >= 0 && (vmin == -__builtin_inff() || (target >= 0 && target <= a.hitH));
    const frac_grid_item rg = a.ranges[r];
    const int i = lane >> 2, g = lane & 3;
    int px[PG];
    int64_t sr2 = 0;
#pragma unroll
    for (int u = 0; u < PG; ++u) {
        const int q = g * PG + u;
        px[u] = (int)a.tgt[(size_t)(rg.y + q / N) * a.tstride + rg.x + (q % N)];
        sr2 += px[u] * px[u];
    }
    sr2 += __shfl_xor(sr2, 1, 64);
    sr2 += __shfl_xor(sr2, 2, 64);
    unsigned long long bestk = kKeyNone;
    const uint32_t vbits = __float_as_uint(vmin);
    for (uint32_t j = 0; j < nent; ++j) { // wave-uniform loop over entries
        const uint2 en = a.entries[(size_t)a.blk_ent[e0 + j / 2] * 64 + col + 32 * (j & 1)];
        if (en.x != vbits)
            continue;
        const int row = (i & 3) + 8 * (i >> 2) + 4 * (int)(j & 1);
        if (!exact) {
            // fp32 fallback regime: every candidate has S16 ≥ 2^24; any valid domain of the
            // bucket routes the range to fallback_fp32 through fit_winner
            const int p = a.tile_pos[en.y * 32 + row];
            const unsigned long long mask = __ballot(p >= 0 && g == 0);
            if (mask) {
                const int pf = __shfl(p, __ffsll((long long)mask) - 1, 64);
                bestk = min(bestk, key_miss((uint64_t)kExactLimit, (uint32_t)pf, 0));
            }
            continue;
        }
        for (uint32_t tile = en.y; tile < min(en.y + (uint32_t)kTilesPerStage, a.ntiles); ++tile) {
            const int p = a.tile_pos[tile * 32 + row];
            unsigned long long tk = kKeyNone;
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const Aff af = lut(t);
                int64_t X = 0;
                if (p >= 0) {
                    const uint32_t* dp = a.pool + (size_t)p * (NN / 2);
#pragma unroll
                    for (int u = 0; u < PG; ++u) {
                        const int f = fwd_rt(af, N, g * PG + u);
                        const uint32_t w = dp[f >> 1];
                        X += (int64_t)px[u] * (int64_t)((f & 1) ? (w >> 16) : (w & 0xffffu));
                    }
                }
                X += __shfl_xor(X, 1, 64);
                X += __shfl_xor(X, 2, 64);
                const int64_t s16 = p >= 0 ? 16 * sr2 - 8 * X - (int64_t)a.negsd2[p] : 0;
                const bool ok = p >= 0 && g == 0 && (hit ? (s16 <= a.hitH) : (s16 == target));
                const unsigned long long mask = __ballot(ok);
                if (mask) {
                    const int first = __ffsll((long long)mask) - 1;
                    const int pf = __shfl(p, first, 64);
                    const unsigned long long k =
                        hit ? key_hit((uint32_t)pf, t) : key_miss((uint64_t)target, (uint32_t)pf, T - 1 - t);
                    tk = k < tk ? k : tk;
                }
            }
            if (tk != kKeyNone) {
                bestk = tk < bestk ? tk : bestk;
                break;
            }
        }
    }
    if (lane == 0)
        a.best_key[r] = bestk;
}

} // namespace fracenc
