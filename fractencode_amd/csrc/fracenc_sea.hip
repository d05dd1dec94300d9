// fracenc_sea.hip — successive-elimination search (FRAC_ENGINE_SEA): the exhaustive search's
// result with most candidates eliminated by a bound that no transform can beat.
//
// For a range R = 4r and a domain's decimated vector D (any of the dihedral transforms permutes
// D's cells, so sums and norms do not depend on t), with SR = ΣR, SD = ΣD and the centred
// norms cR = ‖R − mean R‖, cD = ‖D − mean D‖:
//
//   S16(t) = ‖R − D_t‖² = (SR − SD)²/n² + ‖R̃ − D̃_t‖² ≥ (SR − SD)²/n² + (cR − cD)² = LB
//
// (the mean term is orthogonal to the centred part; the reverse triangle inequality bounds
// the rest).  A candidate can win (or tie) only if S16 ≤ S16* (the range's least error) or it
// is a hit (S16 ≤ H, encode/transformmatcher.h:55,65).  Every domain with LB > max(U, H) for
// some U ≥ S16* is therefore skipped without changing the result: all candidates that reach
// the minimum or a hit are evaluated exactly, and the winner is the least selection key over
// them — the same key the exhaustive engines minimise (fracenc_common.h), so ties resolve to
// the earliest domain and the later transform exactly as TransformEstimator2::estimate
// (encode/TransformEstimator2.hpp:29-48) does.
//
// Layout: the domains of each classifier bucket are sorted by SD (rocPRIM radix sort; the
// pool itself keeps the reference's domain order, so selection keys keep their meaning) into
// 16-byte entries {cD, SD, pool position}.  One wave per range (ranges processed in SR order
// for cache locality): binary search for SR, then 64 candidates per step outward from it,
// LB tested per lane in FP64 (margin 0.5 below the integer S16: conservative), survivors
// compacted through LDS and evaluated exactly in groups of 64/G (lane = candidate row ×
// pixel slice, v_dot2_u32_u16 against G-way sliced inverse-permuted range copies, as
// resolve_dft), the wave's least key then tightens U.  A side closes once the mean term alone
// exceeds the bound (SD is monotone along the sorted order).  Data-dependent: on smooth or
// natural frames ≈0.1–1 % of the candidates are evaluated; on i.i.d. noise it degrades
// towards the exhaustive cost (the bound is never tight).
#include <hipcub/hipcub.hpp>

#include "fracenc_common.h"

namespace fracenc {

constexpr int kSeaMaxBuckets = 8;

struct SeaEntry {
    double cd;    // centred norm of D4
    uint32_t sd;  // ΣD4
    uint32_t pos; // pool position
};
static_assert(sizeof(SeaEntry) == 16, "one dwordx4 per candidate test");

// per pool position: sort key (bucket << 17 | ΣD4) and the position itself
template <int N>
__global__ void __launch_bounds__(256) sea_domain_keys(const uint32_t* __restrict__ pool, uint32_t P,
                                                       const uint32_t* __restrict__ bucket_end, uint32_t nb,
                                                       uint32_t* __restrict__ key, uint32_t* __restrict__ pos)
{
    constexpr int K2 = N * N / 2;
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P)
        return;
    uint32_t sd = 0;
#pragma unroll
    for (int k = 0; k < K2; ++k) {
        const uint32_t w = pool[(size_t)p * K2 + k];
        sd += (w & 0xffffu) + (w >> 16);
    }
    uint32_t b = 0;
    while (b + 1 < nb && p >= bucket_end[b])
        ++b;
    key[p] = (b << 17) | sd; // ΣD4 ≤ 64·1020 < 2^17
    pos[p] = p;
}

// sorted (key, pos) → entries {cD, SD, pos}, and in the same order the pool rows (spool: a
// window of candidates is a contiguous stretch of memory shared by ranges of similar ΣR) and
// −ΣD4² (snegsd2).
// One thread per (entry, 16-byte piece of its row).
template <int N>
__global__ void __launch_bounds__(256) sea_domain_entries(const uint32_t* __restrict__ key,
                                                          const uint32_t* __restrict__ pos,
                                                          const int32_t* __restrict__ negsd2,
                                                          const uint32_t* __restrict__ pool, uint32_t P,
                                                          SeaEntry* __restrict__ ent, uint32_t* __restrict__ spool,
                                                          int32_t* __restrict__ snegsd2)
{
    constexpr int64_t NN = N * N;
    constexpr uint32_t K2 = N * N / 2, PIECES = (K2 + 3) / 4;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= P * PIECES)
        return;
    const uint32_t i = gid / PIECES, piece = gid % PIECES;
    const uint32_t p = pos[i];
    for (uint32_t k = 4 * piece; k < min(4 * piece + 4, K2); ++k)
        spool[(size_t)i * K2 + k] = pool[(size_t)p * K2 + k];
    if (piece)
        return;
    const int64_t sd = key[i] & 0x1ffffu, qd = -(int64_t)negsd2[p];
    SeaEntry e;
    e.cd = sqrt((double)(NN * qd - sd * sd) / (double)NN); // NN·ΣD² − (ΣD)² ≥ 0 exactly
    e.sd = (uint32_t)sd;
    e.pos = p;
    ent[i] = e;
    snegsd2[i] = negsd2[p];
}

// per range: sort key ΣR = 4Σr (range order for locality only)
template <int N>
__global__ void __launch_bounds__(256) sea_range_keys(const uint8_t* __restrict__ tgt, uint32_t tstride,
                                                      const frac_grid_item* __restrict__ ranges, uint32_t nr,
                                                      uint32_t* __restrict__ key, uint32_t* __restrict__ idx)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nr)
        return;
    const frac_grid_item rg = ranges[r];
    uint32_t s = 0;
    for (int y = 0; y < N; ++y)
#pragma unroll
        for (int x = 0; x < N; ++x)
            s += tgt[(size_t)(rg.y + y) * tstride + rg.x + x];
    key[r] = 4u * s;
    idx[r] = r;
}

struct SeaArgs {
    const uint8_t* tgt;
    uint32_t tstride;
    const frac_grid_item* ranges;
    const uint2* rbucket;     // [nr] the range's pool segment [begin, end) (= sorted segment)
    const uint32_t* rorder;   // [nr] ranges in ΣR order
    const SeaEntry* ent;      // [P] per bucket sorted by ΣD4
    const uint32_t* spool;    // [P][n²/2] pool rows in entry order
    const int32_t* snegsd2;   // [P] −ΣD4² in entry order
    uint32_t nr;
    int64_t hitH;             // −1: no hits
    unsigned long long* best_key; // [nr]
    unsigned long long* evaluated; // Σ candidates evaluated exactly (frac_stats.evaluated_mappings)
};

constexpr uint32_t kSeaSeed = 16;  // first step: the 16 candidates nearest in ΣD4 seed the bound
constexpr uint32_t kSeaStep = 128; // later steps: two candidates per lane

template <int N, int T>
__global__ void __launch_bounds__(256) sea_search(SeaArgs a)
{
    constexpr int NN = N * N;
    constexpr int G = NN >= 16 ? 4 : 2; // pixel slices per candidate
    constexpr int R = 64 / G;           // candidates per exact-evaluation group
    constexpr int C = NN / G;           // cells per slice
    constexpr int W = C / 2;            // packed words per slice
    static_assert(C % 2 == 0 && NN <= 64, "n ∈ {2, 4, 8}");
    // survivors of the current step: sorted index, pool position (for the key), −ΣD4²
    __shared__ uint32_t l_idx[4][kSeaStep];
    __shared__ uint32_t l_pos[4][kSeaStep];
    __shared__ int32_t l_nsd[4][kSeaStep];
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t w = blockIdx.x * 4u + wv;
    const int lane = threadIdx.x & 63;
    if (w >= a.nr)
        return;
    const uint32_t r = a.rorder[w];
    const uint2 seg = a.rbucket[r];
    if (seg.x >= seg.y) {
        if (lane == 0)
            a.best_key[r] = kKeyNone;
        return;
    }
    const frac_grid_item rg = a.ranges[r];
    const int rv = lane < NN ? (int)a.tgt[(size_t)(rg.y + lane / N) * a.tstride + rg.x + (lane % N)] : 0;
    int sr = rv, sr2 = rv * rv;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sr += __shfl_xor(sr, o, 64);
        sr2 += __shfl_xor(sr2, o, 64);
    }
    const int64_t SR = 4 * (int64_t)sr, QR = 16 * (int64_t)sr2;
    const double cr = sqrt((double)(NN * QR - SR * SR) / (double)NN);
    const int i = lane / G, g = lane % G;
    uint32_t pk[T][W];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int k = g * C + 2 * j;
            const uint32_t lo = (uint32_t)__shfl(rv, inv_index<N>(t, k), 64);
            const uint32_t hi = (uint32_t)__shfl(rv, inv_index<N>(t, k + 1), 64);
            pk[t][j] = lo | (hi << 16);
        }

    // lower bound of ΣR in the bucket's sorted ΣD: 64-way search, then a ballot
    uint32_t lo = seg.x, hi = seg.y; // answer in [lo, hi]
    while (hi - lo > 64) {
        const uint32_t m = lo + (uint32_t)(((uint64_t)(hi - lo) * (uint32_t)(lane + 1)) / 65u);
        const bool less = (int64_t)a.ent[m].sd < SR;
        const int cnt = __popcll(__ballot(less)); // probes are increasing: the first cnt are "less"
        const uint32_t nlo = cnt ? (uint32_t)__shfl((int)m, cnt - 1, 64) + 1u : lo;
        const uint32_t nhi = cnt < 64 ? (uint32_t)__shfl((int)m, cnt, 64) : hi;
        lo = nlo;
        hi = nhi;
    }
    {
        const uint32_t m = lo + (uint32_t)lane;
        const bool less = m < hi && (int64_t)a.ent[m].sd < SR;
        lo += (uint32_t)__popcll(__ballot(less));
    }

    const double H = a.hitH >= 0 ? (double)a.hitH : -1.0;
    double bound = __builtin_inf(); // max(U, H): candidates with LB above it cannot win
    unsigned long long bestk = kKeyNone;
    uint32_t nevals = 0;
    uint32_t L = lo, Rt = lo; // visited [L, Rt)
    bool lopen = L > seg.x, ropen = Rt < seg.y;
    // the window of a step: up to `want` candidates split over the open sides
    auto plan = [&](uint32_t want, uint32_t cl, uint32_t cr_, bool lo_, bool ro_, uint32_t& nl, uint32_t& nrt) {
        nl = lo_ ? (ro_ ? want / 2 : want) : 0u;
        nl = min(nl, cl - seg.x);
        nrt = ro_ ? min(want - nl, seg.y - cr_) : 0u;
        if (lo_ && nl + nrt < want) // right side short: take more from the left
            nl = min(want - nrt, cl - seg.x);
    };
    // candidate slot k of a step [L − nl, L) ∪ [Rt, Rt + nrt)
    auto slot = [&](uint32_t k, uint32_t cl, uint32_t cr_, uint32_t nl) { return k < nl ? cl - nl + k : cr_ + (k - nl); };
    uint32_t nl, nrt;
    plan(kSeaSeed, L, Rt, lopen, ropen, nl, nrt);
    // per lane: step slots lane and lane + 64
    SeaEntry e[2];
    int32_t en[2];
    uint32_t ix[2];
    bool ev[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const uint32_t k = (uint32_t)lane + 64u * u;
        ev[u] = k < nl + nrt;
        ix[u] = ev[u] ? slot(k, L, Rt, nl) : seg.x;
        e[u] = a.ent[ix[u]];
        en[u] = a.snegsd2[ix[u]];
    }
    while (nl + nrt) {
        // bound test, survivors compacted into the wave's LDS lists
        int ns = 0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            bool surv = false;
            if (ev[u]) {
                const double dm = (double)(SR - (int64_t)e[u].sd), dc = cr - e[u].cd;
                surv = dm * dm * (1.0 / NN) + dc * dc <= bound + 0.5; // 1/n² exact
            }
            const unsigned long long sm = __ballot(surv);
            const int rank = ns + __popcll(sm & ((1ull << lane) - 1ull));
            if (surv) {
                l_idx[wv][rank] = ix[u];
                l_pos[wv][rank] = e[u].pos;
                l_nsd[wv][rank] = en[u];
            }
            ns += __popcll(sm);
        }
        __builtin_amdgcn_wave_barrier();
        nevals += (uint32_t)ns;
        // speculative prefetch of the next step (sides assumed to stay open) and of the entries
        // just outside the window that decide whether they do
        const uint32_t L1 = L - nl, R1 = Rt + nrt;
        const uint32_t sdl = L1 > seg.x ? a.ent[L1 - 1].sd : 0u;
        const uint32_t sdr = R1 < seg.y ? a.ent[R1].sd : 0u;
        uint32_t snl, snr;
        plan(kSeaStep, L1, R1, L1 > seg.x, R1 < seg.y, snl, snr);
        SeaEntry ne[2];
        int32_t nen[2];
        uint32_t nix[2];
        bool nev[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const uint32_t k = (uint32_t)lane + 64u * u;
            nev[u] = k < snl + snr;
            nix[u] = nev[u] ? slot(k, L1, R1, snl) : seg.x;
            ne[u] = a.ent[nix[u]];
            nen[u] = a.snegsd2[nix[u]];
        }

        unsigned long long lk = kKeyNone;
        for (int g0 = 0; g0 < ns; g0 += 2 * R) { // two groups per pass: their loads overlap
            uint32_t dv[2][W];
            uint32_t pp[2];
            int nsd2[2];
            bool have[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int s = g0 + u * R + i;
                have[u] = s < ns;
                const int sl = have[u] ? s : 0;
                const uint32_t si = have[u] ? l_idx[wv][sl] : seg.x;
                pp[u] = l_pos[wv][sl];
                nsd2[u] = l_nsd[wv][sl];
                const uint32_t* dp = a.spool + (size_t)si * (NN / 2) + g * W;
                if constexpr (W % 4 == 0) {
#pragma unroll
                    for (int j = 0; j < W; j += 4) {
                        const uint4 q = *reinterpret_cast<const uint4*>(dp + j);
                        dv[u][j] = q.x, dv[u][j + 1] = q.y, dv[u][j + 2] = q.z, dv[u][j + 3] = q.w;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < W; ++j)
                        dv[u][j] = dp[j];
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                // per transform S16·8 + (T − 1 − t): the least is the candidate's miss order
                // (least error, then the later transform); a hit takes the first t instead
                uint32_t m = ~0u, hitt = (uint32_t)T;
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    uint32_t X = 0;
#pragma unroll
                    for (int j = 0; j < W; ++j)
                        X = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, pk[t][j]),
                                                   __builtin_bit_cast(ushort2_t, dv[u][j]), X, false);
                    X += (uint32_t)__shfl_xor((int)X, 1, 64);
                    if constexpr (G == 4)
                        X += (uint32_t)__shfl_xor((int)X, 2, 64);
                    // S16 = 16Σr² − 8X + ΣD4² ≤ 64·1020² < 2^27: exact in int32, ×8 fits u32
                    const int32_t s16 = 16 * sr2 - 8 * (int32_t)X - nsd2[u];
                    m = min(m, ((uint32_t)s16 << 3) | (uint32_t)(T - 1 - t));
                    if ((int64_t)s16 <= a.hitH && hitt == (uint32_t)T)
                        hitt = (uint32_t)t;
                }
                const unsigned long long key = hitt < (uint32_t)T ? key_hit(pp[u], hitt)
                                                                  : key_miss(m >> 3, pp[u], m & 7u);
                if (have[u] && key < lk)
                    lk = key;
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long ok = __shfl_xor(lk, o, 64);
            lk = ok < lk ? ok : lk;
        }
        if (lk < bestk) {
            bestk = lk;
            if (bestk < kKeyMiss) // a hit: only earlier hits (S16 ≤ H) can still win
                bound = H;
            else
                bound = fmax((double)((bestk & ~kKeyMiss) >> 27), H);
        }
        L = L1;
        Rt = R1;
        // a side closes once the mean term alone exceeds the bound (ΣD4 is monotone along it)
        const double dl = (double)(SR - (int64_t)sdl), dr = (double)((int64_t)sdr - SR);
        lopen = L > seg.x && dl * dl * (1.0 / NN) <= bound + 0.5;
        ropen = Rt < seg.y && dr * dr * (1.0 / NN) <= bound + 0.5;
        plan(kSeaStep, L, Rt, lopen, ropen, nl, nrt);
        if (nl == snl && nrt == snr) { // the usual case: the prefetch was the right window
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                e[u] = ne[u];
                en[u] = nen[u];
                ix[u] = nix[u];
                ev[u] = nev[u];
            }
        } else {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint32_t k = (uint32_t)lane + 64u * u;
                ev[u] = k < nl + nrt;
                ix[u] = ev[u] ? slot(k, L, Rt, nl) : seg.x;
                e[u] = a.ent[ix[u]];
                en[u] = a.snegsd2[ix[u]];
            }
        }
    }
    if (lane == 0) {
        a.best_key[r] = bestk;
        atomicAdd(a.evaluated, (unsigned long long)nevals);
    }
}

} // namespace fracenc
