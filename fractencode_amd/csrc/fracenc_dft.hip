// fracenc_dft.hip — rotation-group (C4) Fourier form of the MFMA search, n = 8, T = 4.
//
// The reference's four transforms (Id, R90, R180, R270; transformmatcher.h:41-45) act on
// the n×n decimated grid as g^t for the single permutation g = fwd(1): fwd(t) = g^t
// (checked at compile time below).  The 64 pixels split into 16 orbits {q, gq, g²q, g³q}
// and with a = r − 128 (range), b = D4 − 512 (domain), per orbit o, k = 0..3:
//
//   Z_t = Σ_p a(p)·b(g^t p) = Σ_o Σ_k a_{o,k}·b_{o,k+t}           (cyclic correlation)
//
// Per orbit let s = x0 + x2, u = x1 + x3, α = a0 − a2, β = a1 − a3, γ = b0 − b2, δ = b1 − b3.
// The length-4 DFT of the correlation gives, with
//   U = Σ(s_a s_b + u_a u_b),  U' = Σ(s_a u_b + u_a s_b),  Pr = Σ(αγ + βδ),  Pi = Σ(βγ − αδ):
//
//   2Z_0 = U + Pr,  2Z_2 = U − Pr,  2Z_1 = U' − Pi,  2Z_3 = U' + Pi
//
// so  2·max_t Z_t = max(U + |Pr|, U' + |Pi|)  and, with S16 = Σ(4r − D4)² = 16Σa² − 8Z + Σb²,
// the chunk statistic tracked per lane is the maximum over domains of
//
//   y = 8·max_t Z_t − Σb²  =  16Σa² − min_t S16                      (one GEMM per tile)
//
// Forms (the tile functions below; the default is the six-MFMA form, kDft6, dft_tile_max6):
//   8-MFMA form  U, U', Pr, Pi as K = 32 GEMMs (8 MFMA 32x32x16 per 32 domains × 32 ranges);
//   five-MFMA    the DFT's real bins P = U + U', M = U − U' (K = 16 each) and the complex bin by
//                Gauss's three products, P ± M on the VALU (kDft5);
//   six-MFMA     the same with M accumulated onto P inside the MFMA (2U, 2U'): 6 MFMA and the
//                exact epilogue's 4.5 VALU per (range, domain) — against the direct form's
//                T·n²/16 = 16 MFMA and 4 transforms × 1.5 VALU.
// Their operand bounds are stated with kDft5 / kDft6; the 8-MFMA form's follow.
//
// Exactness of the 8-MFMA form (f16 operands, f32 accumulate, all values integers):
//   operands  |s_a|,|u_a| ≤ 256, |4s_a| ≤ 1024, |α|,|β| ≤ 255; |s_b|,|u_b| ≤ 1024,
//             |γ|,|δ| ≤ 1020 — integers of magnitude ≤ 2048 are exact in f16;
//   products  every partial sum of U, U' (32 terms ≤ 2^18) and Pr, Pi (32 terms ≤ 2^18) is
//             an integer of magnitude ≤ 2^23: exact in any accumulation order.
//   fast path (per (range block, domain tile) guard 4·max R1·max D∞ + max Σb² ≤ 2^24, with
//             R1 = Σ_o(|s_a| + |u_a|) and D∞ = max_o(|s_b|, |u_b|); ≈93 % of tile pairs on S1):
//             the MFMA starts from C = −Σb² and accumulates 4U (range operands ×4), every
//             partial sum bounded by the guard, so Ũ = 4U − Σb² is exact; then
//             y = max(fma(|Pr|, 4, Ũ), fma(|Pi|, 4, Ũ'))  — 2 fma + a shared v_max3.
//   exact path (guard fails): U, U' from C = 0; 2max Z = max(U + |Pr|, U' + |Pi|) (≤ 2^23,
//             exact); y = fma(that, 4, −Σb²).
//   Both:     y is exact whenever |y| ≤ 2^24, which holds for every candidate in the exact
//             regime S16 < 2^24 (y = 16Σa² − S16, 16Σa² ≤ 2^24).  Candidates with S16 ≥ 2^24
//             may round, but rounding is monotone: their y ≤ 16Σa² − 2^24 (exactly
//             representable) stays ≤ it, so they never beat or tie an exact-regime candidate,
//             and a range whose maximum reaches that bound goes to the fp32 fallback
//             (App. A.3), as with the direct engine.
// The per-lane chunk maximum of y and the tile it appeared in feed resolve_dft, which
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

// T = 8 on the Fourier path: Flip_Rotate_k = Flip ∘ Rotate_k and Flip ∘ Rotate_k ∘ Flip = Rotate_{−k}
template <int N>
constexpr bool flips_valid()
{
    for (int k = 0; k < 4; ++k)
        for (int p = 0; p < N * N; ++p) {
            if (fwd_index<N>(4 + k, p) != fwd_index<N>(4, fwd_index<N>(k, p)))
                return false;
            if (fwd_index<N>(4, fwd_index<N>(k, fwd_index<N>(4, p))) != fwd_index<N>((4 - k) & 3, p))
                return false;
        }
    return true;
}
static_assert(flips_valid<8>(), "the flip half of T = 8 is the rotation search of the flipped range");
constexpr Orbits4<8> kOrb8 = make_orbits4<8>();
constexpr float kDftPadY = -1.0e30f; // −Σb² of padding rows: y ≈ −1e30 never wins
constexpr int kDftRangeFrags = 7;     // s, u, 4s, 4u, α, β, −α

// VAR bit of search_dft: the five-MFMA form (DC / Nyquist bins + a three-product complex bin).
// The length-4 DFT of the per-orbit correlation has two real bins and one complex bin, so with
// P = Σ(s_a + u_a)(s_b + u_b) = U + U' and M = Σ(s_a − u_a)(s_b − u_b) = U − U' (one K = 16
// GEMM each) and the complex bin Pr + iPi = Σ(α + iβ)(γ − iδ) by Gauss's three products
//   k1 = Σγ(α + β),  Pr = k1 + Σ(γ − δ)(−β),  Pi = k1 + Σ(−δ − γ)α
// (the last two accumulate onto k1 inside the MFMA), a tile pair costs 5 MFMA 32x32x16
// instead of 8.  The range operands of the complex bin are doubled so that
//   y = fma(max(P + M + |2Pr|, P − M + |2Pi|), 2, −Σb²)   (= 4·max(U + |Pr|, U' + |Pi|) − Σb²).
// Exactness (a ∈ [−128, 127], b ∈ [−512, 508]; every value an integer):
//   operands  |s_b ± u_b|, |γ − δ|, |δ + γ| ≤ 2048, |γ| ≤ 1020; |s_a ± u_a| ≤ 512,
//             |2(α + β)| ≤ 1020, |2α|, |2β| ≤ 510: exact in f16;
//   P         partial sums ≤ 16·512·2048 = 2^24; M ≤ 16·510·2040 < 2^24: exact;
//   2Pr, 2Pi  partial sums ≤ 2·(16·510·1020 + 16·255·2040) = 33,292,800 < 2^25, all even: exact;
//   P ± M     = 2U, 2U' (|·| ≤ 2^24): exact; + |2Pr| = 4·max(Z_0, Z_2) (≤ 2^24): exact;
//   y         one rounding, exact whenever |y| ≤ 2^24 — the exact-form argument below.
constexpr int kDft5 = 2048;
constexpr int kDftScalar = 4096; // with kDft5: the P ± M and the fma one row per instruction
constexpr int kDft6 = 8192;      // the six-MFMA form (dft_tile_max6)
constexpr int kDftFast6 = 16384; // with kDft6: the guarded constant-folded epilogue (dft_tile_max6_fast)
// issue-cost knobs of the search loop (A/B): the 4-tile chunk unrolled (LDS reads at immediate
// offsets from one base), the stage's LDS-DMA by buffer_load … lds (the stage base in an SGPR
// soffset, per-thread offsets fixed: no VALU per piece), waves of the second half at s_setprio 1
// Row constants of a Fourier tile: [2][16] f32 = 8 uint4, padded to kDftCS = 16 uint4 per tile in
// memory and in the LDS stage, so a 4-tile stage's constants are exactly one 1 KiB LDS-DMA piece
constexpr uint32_t kDftCS = 16;
constexpr int kDftUnroll = 32768;
constexpr int kDftBufDma = 65536;
constexpr int kDftPrio = 131072;

// The five- and six-MFMA forms track h = y/2 = 4·max_t Z_t − Σb²/2 instead of y: the row constant
// (dconst) is −Σb²/2 — exact in f32 (Σb² ≤ 2^24, so a half-integer of magnitude ≤ 2^23) — and the
// epilogue adds it instead of an fma by 2.  The entries keep y (= 2h, exact: a power-of-two scale),
// so resolve_dft and the SEA tiled form read them unchanged.
//
// The guarded fast path of the six-MFMA form (kDftFast6) starts the P GEMM from C = −Σb²/2, so
// both accumulators built on P carry the constant: u' = 2U − Σb²/2, v' = 2U' − Σb²/2, and
//   h = max(u' + |2Pr|, v' + |2Pi|)      — 2 v_add + 1 v_max3 per candidate instead of 4.5 VALU.
// Exactness: every partial sum of u', v' (C included, any accumulation order) is a half-integer of
// magnitude ≤ Σb²/2 + Σ_o(|A0||B0| + |A2||B2|) ≤ Σb²/2 + R6·D6, with R6 = Σ_o(|s_a + u_a| + |s_a − u_a|)
// per range and D6 = max_o max(|s_b + u_b|, |s_b − u_b|) per domain; f32 holds every half-integer
// below 2^23, so the partial sums are exact whenever 2·R6·D6 + Σb² < 2^24.  The guard is taken per
// (range block, domain tile) from the block's max R6 (rguard) and the tile's max 2·D6 and max Σb²
// (tguard); a tile pair that fails it runs the exact epilogue.  2Pr, 2Pi are exact as in kDft5, and
// u' + |2Pr| = 4·max(Z_0, Z_2) − Σb²/2 is one rounding of exact operands — the exact-form argument
// (exact in the exact regime, monotone beyond it) holds unchanged.
constexpr int64_t kFast6Limit = (1ll << 24) - 1; // 2·R6·D6 + Σb² ≤ this

// the form the SEA engine's tiled search (fracenc_tp.hip) runs: 4 or 6
constexpr int kDftTpForm = 6;

template <int VAR>
struct DftForm {
    static constexpr bool F5 = (VAR & kDft5) != 0;
    static constexpr bool F6 = (VAR & kDft6) != 0;
    static constexpr bool FAST6 = F6 && (VAR & kDftFast6) != 0;
    static constexpr bool HALF = F5 || F6;                        // tracks h = y/2 (row constant −Σb²/2)
    static constexpr int KS = (F5 || F6) ? 5 : 4;                 // domain fragments per tile
    static constexpr int NBF = F6 ? 6 : F5 ? 5 : kDftRangeFrags; // range fragments per block
};

struct DftArgs {
    MfmaSearchArgs m;
    uint32_t* rguard;     // [nblocks]  max over the block's ranges of R1 = Σ_o(|s_a| + |u_a|) (six-MFMA
                          //            form: R6 = Σ_o(|s_a + u_a| + |s_a − u_a|))
    uint2* tguard;        // [ntiles]   {max 4·D∞, max Σb²} over the tile's valid rows (five- / six-MFMA
                          //            layout: {max 2·D6, max Σb²})
    const uint32_t* choff; // CHUNKED: [work] first chunk entry of the work item (fracenc_tp.hip)
    const int32_t* trmax;  // kDftFast6: [ntiles] the largest block R6 whose guard holds against the
                           // tile, (kFast6Limit − max Σb²) / max 2·D6 (−1: none)
    unsigned long long* stamps = nullptr; // FRAC_CLOCK_STAMP builds only: [workgroups][kClockStampWords]
    // not CHUNKED: per range slot the maximum over every work item, merged here with one 64-bit atomicMax per
    // (slot, work item) instead of per-work-item entries: fmap(y) << 32 | (kSlotBestTileMax − chunk) << 6 |
    // the chunk's tiles to re-evaluate << 2 | the lane halves of that chunk attaining y.  The greatest word names
    // the greatest y and, among equal y, the earliest chunk — the chunk resolve_dft walked the entries for.  The
    // tile mask is 0xf unless the search tracked the tiles attaining y (TMASK); 0 = no work item reached the slot.
    unsigned long long* slotbest = nullptr;
};
constexpr uint32_t kSlotBestTileMax = 0x3ffffffu; // chunk tiles below 2^26 (domains < 2^24: tiles < 2^19)
// per workgroup: s_memtime and s_memrealtime before / after the loop, HW_ID | XCC_ID << 32, and the
// work item's tile range first | end << 32
constexpr uint32_t kClockStampWords = 6;

// ---------------------------------------------------------------------------
// dft_domain_build: pool_build + dft_domain_prep in one pass for the Fourier path.  One
// thread per (tile, row) = per pool position: the 2×2 sums come straight from the plane
// (SamplerBilinear's integer sum, image/sampler.h:21-38, as pool_build), two cells per
// 32-bit word — (w & 0x00ff00ff) + ((w >> 8) & 0x00ff00ff) over the word of both rows is
// the packed u16 pair the pool stores — and the same registers feed the tile fragments.
// Outputs: the pool and −ΣD4² (read by fit_winner and fallback_grid), the pool rows again in
// tile order (resolve_dft); per 32-domain tile the A fragments of the four K-steps
// [s_b | u_b | γ | δ] (lane l: row l&31, orbit 8(l>>5) + j), −Σb² per row in the [2][16]
// lane-half layout of the epilogue, and the tile's fast-path guard terms.  Every pool
// position sits in exactly one tile row.
// ---------------------------------------------------------------------------
struct DftDomainBuildArgs {
    const uint8_t* src;
    uint32_t sstride;
    const frac_grid_item* doms;
    const uint32_t* porig;      // pool position → domain index
    uint32_t* pool;             // [P][32] packed u16 pairs of D4
    int32_t* negsd2;            // [P]
    uint32_t* tpool;            // [ntiles*32][32] the same rows in tile order, orbit order (resolve_dft)
    const uint32_t* row_of = nullptr; // BYPOS: [P] tile row of each pool position (tp_build_tiles)
    uint32_t npos = 0;                // BYPOS: P
};

// pair_sums: fracenc_kernels.hip (pool_build)

// BYPOS (the SEA tiled form, whose tiles hold domains in ΣD4 order): one thread per pool
// position in domain order, so neighbouring threads read overlapping plane rows, and the
// outputs are scattered to the position's tile row; tp_build_tiles writes the padding rows and
// zeroes the tile guards, which are then raised with atomics.
// F5: the five-MFMA form's fragments [s_b + u_b | s_b − u_b | γ | γ − δ | −δ − γ] (kDft5)
template <bool BYPOS = false, bool F5 = false>
__device__ __forceinline__ void dft_domain_build_at(uint32_t tid, const MfmaDomainPrepArgs& a, const DftDomainBuildArgs& s,
                                                    uint2* __restrict__ tguard, int32_t* __restrict__ trmax)
{
    constexpr int NN = 64, NO = 16, KS = F5 ? 5 : 4;
    if (tid >= (BYPOS ? s.npos : a.ntiles * 32u))
        return;
    const uint32_t gid = BYPOS ? s.row_of[tid] : tid;
    const uint32_t tile = gid >> 5, row = gid & 31u;
    const int p = BYPOS ? (int)tid : a.tile_pos[gid];
    uint32_t w[NN / 2];
    if (p >= 0) {
        const frac_grid_item d = s.doms[s.porig[p]];
        const uint8_t* base = s.src + (size_t)d.y * s.sstride + d.x;
        if ((((uintptr_t)base | s.sstride) & 7u) == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                // 16 bytes per row: two 8-byte loads (domain origins are 8-byte aligned, not 16)
                const uint2* r0 = reinterpret_cast<const uint2*>(base + (size_t)(2 * i) * s.sstride);
                const uint2* r1 = reinterpret_cast<const uint2*>(base + (size_t)(2 * i + 1) * s.sstride);
                const uint2 a0 = r0[0], a1 = r0[1], b0 = r1[0], b1 = r1[1];
                w[4 * i + 0] = pair_sums(a0.x, b0.x);
                w[4 * i + 1] = pair_sums(a0.y, b0.y);
                w[4 * i + 2] = pair_sums(a1.x, b1.x);
                w[4 * i + 3] = pair_sums(a1.y, b1.y);
            }
        } else {
#pragma unroll
            for (int k = 0; k < NN / 2; ++k) {
                const uint8_t* q = base + (size_t)(2 * (k / 4)) * s.sstride + 4 * (k % 4);
                const uint32_t w0 = q[0] | (q[1] << 8) | (q[2] << 16) | ((uint32_t)q[3] << 24);
                const uint8_t* q1 = q + s.sstride;
                const uint32_t w1 = q1[0] | (q1[1] << 8) | (q1[2] << 16) | ((uint32_t)q1[3] << 24);
                w[k] = pair_sums(w0, w1);
            }
        }
        uint4* pw = reinterpret_cast<uint4*>(s.pool + (size_t)p * (NN / 2));
        int sq = 0;
#pragma unroll
        for (int k = 0; k < NN / 2; ++k) {
            const int lo = (int)(w[k] & 0xffffu), hi = (int)(w[k] >> 16);
            sq += lo * lo + hi * hi;
        }
#pragma unroll
        for (int k = 0; k < NN / 8; ++k)
            pw[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
        // the tile-order copy for resolve_dft, orbit o as (D_{o,0} | D_{o,1} << 16), (D_{o,2} | D_{o,3} << 16)
        auto cell = [&](int q) { return (w[q >> 1] >> (16 * (q & 1))) & 0xffffu; };
        uint4* tw = reinterpret_cast<uint4*>(s.tpool + (size_t)gid * (NN / 2));
#pragma unroll
        for (int v = 0; v < NN / 8; ++v) {
            uint32_t d[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = 2 * v + (e >> 1), k = 2 * (e & 1);
                d[e] = cell(kOrb8.p[o][k]) | (cell(kOrb8.p[o][k + 1]) << 16);
            }
            tw[v] = make_uint4(d[0], d[1], d[2], d[3]);
        }
        s.negsd2[p] = -sq;
    } else {
#pragma unroll
        for (int k = 0; k < NN / 2; ++k)
            w[k] = 0x02000200u; // padding: b = 0
    }
    int b[NN];
    int sb2 = 0;
#pragma unroll
    for (int k = 0; k < NN / 2; ++k) {
        b[2 * k] = (int)(w[k] & 0xffffu) - 512;
        b[2 * k + 1] = (int)(w[k] >> 16) - 512;
    }
#pragma unroll
    for (int k = 0; k < NN; ++k)
        sb2 += b[k] * b[k];
    _Float16 comp[KS][NO];
    int dinf = 0;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
        const int b0 = b[kOrb8.p[o][0]], b1 = b[kOrb8.p[o][1]], b2 = b[kOrb8.p[o][2]], b3 = b[kOrb8.p[o][3]];
        const int sb = b0 + b2, ub = b1 + b3, gb = b0 - b2, db = b1 - b3;
        // guard term: D∞ = max(|s_b|, |u_b|) (8-MFMA form); D6 = max(|s_b + u_b|, |s_b − u_b|) (F5 layout)
        dinf = F5 ? max(dinf, max(abs(sb + ub), abs(sb - ub))) : max(dinf, max(abs(sb), abs(ub)));
        if constexpr (F5) {
            comp[0][o] = (_Float16)(sb + ub);
            comp[1][o] = (_Float16)(sb - ub);
            comp[2][o] = (_Float16)gb;
            comp[3][o] = (_Float16)(gb - db);
            comp[4][o] = (_Float16)(-db - gb);
        } else {
            comp[0][o] = (_Float16)sb;
            comp[1][o] = (_Float16)ub;
            comp[2][o] = (_Float16)gb;
            comp[3][o] = (_Float16)db;
        }
    }
#pragma unroll
    for (int st = 0; st < KS; ++st)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            _Float16 v8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                v8[j] = comp[st][8 * h + j];
            a.dtiles[((size_t)tile * KS + st) * 64 + row + 32 * h] = __builtin_bit_cast(uint4, v8);
        }
    // the row constant: −Σb² (8-MFMA form, tracks y), −Σb²/2 (F5 layout: the five- and six-MFMA
    // forms track h = y/2; exact, Σb² ≤ 2^24)
    const float ny = p >= 0 ? (F5 ? -0.5f * (float)sb2 : -(float)sb2) : kDftPadY;
    const uint32_t h = (row >> 2) & 1u, i = (row & 3u) + 4u * (row >> 3);
    a.dconst[(size_t)tile * (kDftCS * 4) + h * 16 + i] = __float_as_uint(ny);
    uint32_t gx = p >= 0 ? (uint32_t)((F5 ? 2 : 4) * dinf) : 0u, gy = p >= 0 ? (uint32_t)sb2 : 0u;
    if constexpr (BYPOS) {
        atomicMax(&tguard[tile].x, gx);
        atomicMax(&tguard[tile].y, gy);
        return;
    }
    // the tile's guard terms over its valid rows: a 32-lane maximum (whole tiles leave together
    // above), one writer per tile
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
        gx = max(gx, (uint32_t)__shfl_xor((int)gx, o, 64));
        gy = max(gy, (uint32_t)__shfl_xor((int)gy, o, 64));
    }
    if (row == 0) {
        tguard[tile] = make_uint2(gx, gy);
        // the six-MFMA fast path's guard as one threshold on the block's R6:
        // R6·gx + gy ≤ kFast6Limit  ⇔  gy ≤ kFast6Limit and R6 ≤ ⌊(kFast6Limit − gy) / gx⌋
        if (F5 && trmax)
            trmax[tile] = (int64_t)gy > kFast6Limit ? -1
                          : gx == 0                  ? INT32_MAX
                                                     : (int32_t)min<int64_t>((kFast6Limit - gy) / gx, INT32_MAX);
    }
}

// dft_domain_build_at restated with two lanes per tile row (dft_prep, round 4): lane h of a row loads
// the plane rows of D4 rows 4h … 4h + 3, writes that half of the pool row, and puts it in LDS; each lane
// then reads the cells of orbits 8h … 8h + 7 back (LDS addresses from the orbit table, no register
// indexing) and builds that lane half of the fragments and of the tile-order copy.  Σb², ΣD4² and the
// guard terms meet in a lane-pair shuffle.  On a small frame the single-thread chain per row ran one
// wave per CU on a quarter of the CUs (C2: 16 workgroups); this halves the chain and doubles the waves.
// A tile's 32 rows are one wave's 64 lanes, so the tile guards stay a wave reduction.
constexpr uint32_t kDbRowWords = 33; // LDS words per row: 32 + 1 of padding (rows in distinct banks)
template <bool F5>
__device__ __forceinline__ void dft_domain_build_pair_at(uint32_t tid2, const MfmaDomainPrepArgs& a,
                                                         const DftDomainBuildArgs& s, uint2* __restrict__ tguard,
                                                         int32_t* __restrict__ trmax)
{
    constexpr int KS = F5 ? 5 : 4;
    __shared__ uint32_t rows[128 * kDbRowWords]; // 256 threads = 128 rows
    const uint32_t gid = tid2 >> 1, hh = tid2 & 1u;
    if (gid >= a.ntiles * 32u) // whole tiles (whole waves) leave together
        return;
    const uint32_t tile = gid >> 5, row = gid & 31u;
    uint32_t* lrow = rows + ((threadIdx.x >> 1) & 127u) * kDbRowWords;
    const int p = a.tile_pos[gid];
    uint32_t w[16]; // words 16hh … 16hh + 15 of the row: D4 rows 4hh … 4hh + 3, two cells per word
    int sq = 0;
    if (p >= 0) {
        const frac_grid_item d = s.doms[s.porig[p]];
        const uint8_t* base = s.src + (size_t)(d.y + 8 * hh) * s.sstride + d.x;
        if ((((uintptr_t)base | s.sstride) & 7u) == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint2* r0 = reinterpret_cast<const uint2*>(base + (size_t)(2 * i) * s.sstride);
                const uint2* r1 = reinterpret_cast<const uint2*>(base + (size_t)(2 * i + 1) * s.sstride);
                const uint2 a0 = r0[0], a1 = r0[1], b0 = r1[0], b1 = r1[1];
                w[4 * i + 0] = pair_sums(a0.x, b0.x);
                w[4 * i + 1] = pair_sums(a0.y, b0.y);
                w[4 * i + 2] = pair_sums(a1.x, b1.x);
                w[4 * i + 3] = pair_sums(a1.y, b1.y);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint8_t* q = base + (size_t)(2 * (k / 4)) * s.sstride + 4 * (k % 4);
                const uint32_t w0 = q[0] | (q[1] << 8) | (q[2] << 16) | ((uint32_t)q[3] << 24);
                const uint8_t* q1 = q + s.sstride;
                const uint32_t w1 = q1[0] | (q1[1] << 8) | (q1[2] << 16) | ((uint32_t)q1[3] << 24);
                w[k] = pair_sums(w0, w1);
            }
        }
        uint4* pw = reinterpret_cast<uint4*>(s.pool + (size_t)p * 32 + 16 * hh);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            pw[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int lo = (int)(w[k] & 0xffffu), hi = (int)(w[k] >> 16);
            sq += lo * lo + hi * hi;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k)
            w[k] = 0x02000200u; // padding: b = 0
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
        lrow[16 * hh + k] = w[k];
    sq += __shfl_xor(sq, 1, 64);
    if (p >= 0 && hh == 0)
        s.negsd2[p] = -sq;
    // the pair's LDS writes above are one wave's and precede its reads below in program order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint16_t* cells = reinterpret_cast<const uint16_t*>(lrow);
    // orbits 8hh … 8hh + 7: their four cells each (the table's entries, selected by the lane half)
    int cv[8][4];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            cv[j][k] = cells[hh ? kOrb8.p[8 + j][k] : kOrb8.p[j][k]];
    if (p >= 0) {
        // the tile-order copy for resolve_dft, orbit o as (D_{o,0} | D_{o,1} << 16), (D_{o,2} | D_{o,3} << 16)
        uint4* tw = reinterpret_cast<uint4*>(s.tpool + (size_t)gid * 32 + 16 * hh);
#pragma unroll
        for (int v = 0; v < 4; ++v)
            tw[v] = make_uint4((uint32_t)cv[2 * v][0] | ((uint32_t)cv[2 * v][1] << 16),
                               (uint32_t)cv[2 * v][2] | ((uint32_t)cv[2 * v][3] << 16),
                               (uint32_t)cv[2 * v + 1][0] | ((uint32_t)cv[2 * v + 1][1] << 16),
                               (uint32_t)cv[2 * v + 1][2] | ((uint32_t)cv[2 * v + 1][3] << 16));
    }
    int sb2 = 0, dinf = 0;
    _Float16 comp[KS][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int b0 = cv[j][0] - 512, b1 = cv[j][1] - 512, b2 = cv[j][2] - 512, b3 = cv[j][3] - 512;
        sb2 += b0 * b0 + b1 * b1 + b2 * b2 + b3 * b3;
        const int sb = b0 + b2, ub = b1 + b3, gb = b0 - b2, db = b1 - b3;
        dinf = F5 ? max(dinf, max(abs(sb + ub), abs(sb - ub))) : max(dinf, max(abs(sb), abs(ub)));
        if constexpr (F5) {
            comp[0][j] = (_Float16)(sb + ub);
            comp[1][j] = (_Float16)(sb - ub);
            comp[2][j] = (_Float16)gb;
            comp[3][j] = (_Float16)(gb - db);
            comp[4][j] = (_Float16)(-db - gb);
        } else {
            comp[0][j] = (_Float16)sb;
            comp[1][j] = (_Float16)ub;
            comp[2][j] = (_Float16)gb;
            comp[3][j] = (_Float16)db;
        }
    }
#pragma unroll
    for (int st = 0; st < KS; ++st)
        a.dtiles[((size_t)tile * KS + st) * 64 + row + 32 * hh] = __builtin_bit_cast(uint4, comp[st]);
    sb2 += __shfl_xor(sb2, 1, 64);
    dinf = max(dinf, __shfl_xor(dinf, 1, 64));
    if (hh == 0) {
        const float ny = p >= 0 ? (F5 ? -0.5f * (float)sb2 : -(float)sb2) : kDftPadY;
        const uint32_t h = (row >> 2) & 1u, i = (row & 3u) + 4u * (row >> 3);
        a.dconst[(size_t)tile * (kDftCS * 4) + h * 16 + i] = __float_as_uint(ny);
    }
    uint32_t gx = p >= 0 ? (uint32_t)((F5 ? 2 : 4) * dinf) : 0u, gy = p >= 0 ? (uint32_t)sb2 : 0u;
    // the tile's guard terms over its 32 rows (lanes 2·row + hh of one wave): a wave maximum
#pragma unroll
    for (int o = 32; o > 1; o >>= 1) {
        gx = max(gx, (uint32_t)__shfl_xor((int)gx, o, 64));
        gy = max(gy, (uint32_t)__shfl_xor((int)gy, o, 64));
    }
    if (row == 0 && hh == 0) {
        tguard[tile] = make_uint2(gx, gy);
        if (F5 && trmax)
            trmax[tile] = (int64_t)gy > kFast6Limit ? -1
                          : gx == 0                  ? INT32_MAX
                                                     : (int32_t)min<int64_t>((kFast6Limit - gy) / gx, INT32_MAX);
    }
}

template <bool BYPOS = false, bool F5 = false>
__global__ void __launch_bounds__(256) dft_domain_build(MfmaDomainPrepArgs a, DftDomainBuildArgs s,
                                                        uint2* __restrict__ tguard, int32_t* __restrict__ trmax = nullptr)
{
    dft_domain_build_at<BYPOS, F5>(blockIdx.x * blockDim.x + threadIdx.x, a, s, tguard, trmax);
}

// ---------------------------------------------------------------------------
// dft_range_prep: per range block the seven distinct B fragments
//   f0 = s_a, f1 = u_a, f2 = 4s_a, f3 = 4u_a, f4 = α, f5 = β, f6 = −α
// (lane l: range slot l&31, orbit 8(l>>5) + j); U = [f0|f1], U' = [f1|f0] (×4: f2, f3),
// Pr = [f4|f5], Pi = [f5|f6] against the domain K-steps [s_b|u_b], [γ|δ].  Also 16Σa² per
// slot and the block's guard term max R1.  One thread per slot (a range-order variant with
// scattered outputs measured slower for the SEA tiled form's ΣR-sorted slots: 61 vs 41 µs).
// ---------------------------------------------------------------------------
// FORM 5: the five-MFMA form's fragments [s_a + u_a | s_a − u_a | 2(α + β) | −2β | 2α] (kDft5);
// FORM 6: the six-MFMA form's [s_a + u_a | s_a − u_a | u_a − s_a | 2(α + β) | −2β | 2α] (kDft6)
template <int FORM = 4>
__device__ __forceinline__ void dft_range_prep_at(uint32_t gid, const MfmaRangePrepArgs& a, uint32_t* __restrict__ rguard)
{
    constexpr int N = 8, NN = 64, NO = 16, NBF = FORM == 6 ? 6 : FORM == 5 ? 5 : kDftRangeFrags;
    if (gid >= a.nblocks * 32u)
        return;
    const uint32_t b = gid >> 5, col = gid & 31u;
    const int ri = a.slot_range[gid];
    int av[NN];
    int sa2 = 0;
    if (ri >= 0) {
        const frac_grid_item rg = a.ranges[ri];
        const uint8_t* base = a.tgt + (size_t)rg.y * a.tstride + rg.x;
        if ((((uintptr_t)base | a.tstride) & 7u) == 0) {
            // one 8-byte load per row (range origins on the 8-pixel grid)
#pragma unroll
            for (int y = 0; y < N; ++y) {
                const uint2 w = *reinterpret_cast<const uint2*>(base + (size_t)y * a.tstride);
#pragma unroll
                for (int x = 0; x < N; ++x)
                    av[y * N + x] = (int)(((x < 4 ? w.x : w.y) >> (8 * (x & 3))) & 0xffu) - 128;
            }
        } else {
#pragma unroll
            for (int q = 0; q < NN; ++q)
                av[q] = (int)base[(size_t)(q / N) * a.tstride + (q % N)] - 128;
        }
#pragma unroll
        for (int q = 0; q < NN; ++q)
            sa2 += av[q] * av[q];
        if (b >= a.flip_from) {
            // T = 8: the block's flipped copy, a'(q) = a(Flip q).  Flip_Rotate_k = Flip ∘ Rotate_k
            // (fwd(4 + k, p) = fwd(4, fwd(k, p)), image/transform.h:32-41) and Flip ∘ g^k ∘ Flip = g^−k, so
            // Σ_p a(p)·b(fwd(4 + k, p)) = Σ_q a'(q)·b(g^{−k} q): the copy's rotation t' is transform 4 + (−t' mod 4)
            int fv[NN];
#pragma unroll
            for (int q = 0; q < NN; ++q)
                fv[q] = av[fwd_index<N>(4, q)];
#pragma unroll
            for (int q = 0; q < NN; ++q)
                av[q] = fv[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < NN; ++q)
            av[q] = 0;
    }
    _Float16 comp[NBF][NO];
    int r1 = 0;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
        const int a0 = av[kOrb8.p[o][0]], a1 = av[kOrb8.p[o][1]], a2 = av[kOrb8.p[o][2]], a3 = av[kOrb8.p[o][3]];
        const int sa = a0 + a2, ua = a1 + a3, al = a0 - a2, be = a1 - a3;
        // guard term: R1 = Σ(|s_a| + |u_a|); the six-MFMA form's R6 = Σ(|s_a + u_a| + |s_a − u_a|)
        r1 += FORM == 6 ? abs(sa + ua) + abs(sa - ua) : abs(sa) + abs(ua);
        if constexpr (FORM == 5) {
            comp[0][o] = (_Float16)(sa + ua);
            comp[1][o] = (_Float16)(sa - ua);
            comp[2][o] = (_Float16)(2 * (al + be));
            comp[3][o] = (_Float16)(-2 * be);
            comp[4][o] = (_Float16)(2 * al);
        } else if constexpr (FORM == 6) {
            comp[0][o] = (_Float16)(sa + ua);
            comp[1][o] = (_Float16)(sa - ua);
            comp[2][o] = (_Float16)(ua - sa);
            comp[3][o] = (_Float16)(2 * (al + be));
            comp[4][o] = (_Float16)(-2 * be);
            comp[5][o] = (_Float16)(2 * al);
        } else {
            comp[0][o] = (_Float16)sa;
            comp[1][o] = (_Float16)ua;
            comp[2][o] = (_Float16)(4 * sa);
            comp[3][o] = (_Float16)(4 * ua);
            comp[4][o] = (_Float16)al;
            comp[5][o] = (_Float16)be;
            comp[6][o] = (_Float16)(-al);
        }
    }
#pragma unroll
    for (int f = 0; f < NBF; ++f)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            _Float16 v8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                v8[j] = comp[f][8 * h + j];
            a.rfrags[((size_t)b * NBF + f) * 64 + col + 32 * h] = __builtin_bit_cast(uint4, v8);
        }
    a.rconst[gid] = ri >= 0 ? (uint32_t)(16 * sa2) : 0u; // 16Σa² ≤ 2^24
    if (a.slotbest)
        a.slotbest[gid] = 0ull; // the run's reset of the search's merged maxima
    if (a.rorb) {
        // raw pixels r = a + 128, orbit o as the pairs (r_{o,0} | r_{o,1} << 16), (r_{o,2} | r_{o,3} << 16)
        uint4* ro = reinterpret_cast<uint4*>(a.rorb + (size_t)gid * 32);
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            uint32_t d[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = 2 * v + (e >> 1), k = 2 * (e & 1);
                d[e] = (uint32_t)(av[kOrb8.p[o][k]] + 128) | ((uint32_t)(av[kOrb8.p[o][k + 1]] + 128) << 16);
            }
            ro[v] = make_uint4(d[0], d[1], d[2], d[3]);
        }
    }
    // the block's guard: a 32-lane maximum (whole blocks leave together above), one writer
    uint32_t g1 = (uint32_t)r1;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1)
        g1 = max(g1, (uint32_t)__shfl_xor((int)g1, o, 64));
    if (col == 0)
        rguard[b] = g1;
}

// dft_range_prep_at restated with two lanes per range slot (dft_prep, round 4), as the domain build: lane h
// loads rows 4h … 4h + 3 of the range into LDS; each lane then reads the pixels of orbits 8h … 8h + 7 back
// (T = 8's flipped copies read through the Flip permutation: the same table, another address) and builds that
// lane half of the fragments and of the orbit-ordered pixel pairs.  Σa² and R6 meet in a lane-pair shuffle;
// a block's 32 slots are one wave, so its guard stays a wave maximum.
template <int FORM>
__device__ __forceinline__ void dft_range_prep_pair_at(uint32_t gid2, const MfmaRangePrepArgs& a,
                                                       uint32_t* __restrict__ rguard)
{
    constexpr int N = 8, NBF = FORM == 6 ? 6 : FORM == 5 ? 5 : kDftRangeFrags;
    constexpr uint32_t kRow = 68; // LDS bytes per slot: 64 + 4 of padding
    __shared__ uint8_t px[128 * kRow];
    const uint32_t gid = gid2 >> 1, hh = gid2 & 1u;
    if (gid >= a.nblocks * 32u) // whole blocks (whole waves) leave together
        return;
    const uint32_t b = gid >> 5, col = gid & 31u;
    uint8_t* lp = px + ((threadIdx.x >> 1) & 127u) * kRow;
    const int ri = a.slot_range[gid];
    uint2 w[4] = {make_uint2(0x80808080u, 0x80808080u), make_uint2(0x80808080u, 0x80808080u),
                  make_uint2(0x80808080u, 0x80808080u), make_uint2(0x80808080u, 0x80808080u)}; // empty: a = 0
    if (ri >= 0) {
        const frac_grid_item rg = a.ranges[ri];
        const uint8_t* base = a.tgt + (size_t)(rg.y + 4 * hh) * a.tstride + rg.x;
        if ((((uintptr_t)base | a.tstride) & 7u) == 0) {
#pragma unroll
            for (int y = 0; y < 4; ++y)
                w[y] = *reinterpret_cast<const uint2*>(base + (size_t)y * a.tstride);
        } else {
#pragma unroll
            for (int y = 0; y < 4; ++y) {
                const uint8_t* q = base + (size_t)y * a.tstride;
                w[y] = make_uint2(q[0] | (q[1] << 8) | (q[2] << 16) | ((uint32_t)q[3] << 24),
                                  q[4] | (q[5] << 8) | (q[6] << 16) | ((uint32_t)q[7] << 24));
            }
        }
    }
    uint32_t* lw = reinterpret_cast<uint32_t*>(lp);
#pragma unroll
    for (int y = 0; y < 4; ++y) {
        lw[8 * hh + 2 * y] = w[y].x;
        lw[8 * hh + 2 * y + 1] = w[y].y;
    }
    // the pair's LDS writes above are one wave's and precede its reads below in program order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // T = 8: the block's flipped copy, a'(q) = a(Flip q) (dft_range_prep_at)
    const bool flip = ri >= 0 && b >= a.flip_from;
    int av[8][4]; // orbits 8hh … 8hh + 7, their four pixels − 128
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q0 = kOrb8.p[j][k], q1 = kOrb8.p[8 + j][k];
            const int q = hh ? q1 : q0, qf = hh ? fwd_index<N>(4, q1) : fwd_index<N>(4, q0);
            av[j][k] = (int)lp[flip ? qf : q] - 128;
        }
    int sa2 = 0, r1 = 0;
    _Float16 comp[NBF][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int a0 = av[j][0], a1 = av[j][1], a2 = av[j][2], a3 = av[j][3];
        sa2 += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
        const int sa = a0 + a2, ua = a1 + a3, al = a0 - a2, be = a1 - a3;
        r1 += FORM == 6 ? abs(sa + ua) + abs(sa - ua) : abs(sa) + abs(ua);
        if constexpr (FORM == 5) {
            comp[0][j] = (_Float16)(sa + ua);
            comp[1][j] = (_Float16)(sa - ua);
            comp[2][j] = (_Float16)(2 * (al + be));
            comp[3][j] = (_Float16)(-2 * be);
            comp[4][j] = (_Float16)(2 * al);
        } else if constexpr (FORM == 6) {
            comp[0][j] = (_Float16)(sa + ua);
            comp[1][j] = (_Float16)(sa - ua);
            comp[2][j] = (_Float16)(ua - sa);
            comp[3][j] = (_Float16)(2 * (al + be));
            comp[4][j] = (_Float16)(-2 * be);
            comp[5][j] = (_Float16)(2 * al);
        } else {
            comp[0][j] = (_Float16)sa;
            comp[1][j] = (_Float16)ua;
            comp[2][j] = (_Float16)(4 * sa);
            comp[3][j] = (_Float16)(4 * ua);
            comp[4][j] = (_Float16)al;
            comp[5][j] = (_Float16)be;
            comp[6][j] = (_Float16)(-al);
        }
    }
    if (ri < 0) { // an empty slot's fragments are zero (its pixels read as 128 above: already so), no guard
        sa2 = 0;
        r1 = 0;
    }
#pragma unroll
    for (int f = 0; f < NBF; ++f)
        a.rfrags[((size_t)b * NBF + f) * 64 + col + 32 * hh] = __builtin_bit_cast(uint4, comp[f]);
    sa2 += __shfl_xor(sa2, 1, 64);
    r1 += __shfl_xor(r1, 1, 64);
    if (hh == 0) {
        a.rconst[gid] = ri >= 0 ? (uint32_t)(16 * sa2) : 0u; // 16Σa² ≤ 2^24
        if (a.slotbest)
            a.slotbest[gid] = 0ull; // the run's reset of the search's merged maxima
    }
    if (a.rorb) {
        // raw pixels r = a + 128, orbit o as the pairs (r_{o,0} | r_{o,1} << 16), (r_{o,2} | r_{o,3} << 16)
        uint4* ro = reinterpret_cast<uint4*>(a.rorb + (size_t)gid * 32 + 16 * hh);
#pragma unroll
        for (int v = 0; v < 4; ++v)
            ro[v] = make_uint4((uint32_t)(av[2 * v][0] + 128) | ((uint32_t)(av[2 * v][1] + 128) << 16),
                               (uint32_t)(av[2 * v][2] + 128) | ((uint32_t)(av[2 * v][3] + 128) << 16),
                               (uint32_t)(av[2 * v + 1][0] + 128) | ((uint32_t)(av[2 * v + 1][1] + 128) << 16),
                               (uint32_t)(av[2 * v + 1][2] + 128) | ((uint32_t)(av[2 * v + 1][3] + 128) << 16));
    }
    // the block's guard: a maximum over its 32 slots (lanes 2·col + hh of one wave), one writer
    uint32_t g1 = (uint32_t)r1;
#pragma unroll
    for (int o = 32; o > 1; o >>= 1)
        g1 = max(g1, (uint32_t)__shfl_xor((int)g1, o, 64));
    if (col == 0 && hh == 0)
        rguard[b] = g1;
}

template <int FORM = 4>
__global__ void __launch_bounds__(256) dft_range_prep(MfmaRangePrepArgs a, uint32_t* __restrict__ rguard)
{
    dft_range_prep_at<FORM>(blockIdx.x * blockDim.x + threadIdx.x, a, rguard);
}

// ---------------------------------------------------------------------------
// dft_prep: the Fourier path's preparation in one launch.  Blocks [0, dblocks) build the domain
// tiles (dft_domain_build), the rest prepare the range blocks (dft_range_prep), so the two run
// side by side instead of one after the other.  Every thread also takes a grid-stride share of
// the run's best_key reset, and thread 0 sets the fallback count: the two hipMemsetAsync of
// launch_all, whose launches cost more than their bytes on small frames.
// ---------------------------------------------------------------------------
struct DftPrepInit {
    unsigned long long* best_key = nullptr; // nr entries set to ~0 (no candidate yet)
    uint32_t nr = 0;
    uint32_t* fb_count = nullptr; // set to fbc when not null
    uint32_t fbc = 0;
    uint32_t dblocks = 0; // blocks of the domain build
    const DevPlan* plan = nullptr; // device-planned search: tile / block / range counts from the plan
    uint32_t copies = 1;           // with a plan: range blocks per planned block (T = 8 Fourier: 2)
};

template <int FORM>
__global__ void __launch_bounds__(256) dft_prep(MfmaDomainPrepArgs d, DftDomainBuildArgs s, uint2* __restrict__ tguard,
                                                int32_t* __restrict__ trmax, MfmaRangePrepArgs r,
                                                uint32_t* __restrict__ rguard, DftPrepInit in)
{
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
    if (in.plan) {
        d.ntiles = in.plan->ntiles;
        apply_plan(r, in.copies);
        in.nr = in.plan->nr;
    }
    for (uint32_t i = gt; i < in.nr; i += gridDim.x * blockDim.x)
        in.best_key[i] = ~0ull;
    if (gt == 0 && in.fb_count)
        *in.fb_count = in.fbc;
    if (blockIdx.x < in.dblocks)
        dft_domain_build_pair_at<FORM != 4>(gt, d, s, tguard, trmax); // two lanes per tile row
    else // two lanes per range slot
        dft_range_prep_pair_at<FORM>((blockIdx.x - in.dblocks) * blockDim.x + threadIdx.x, r, rguard);
}

// ---------------------------------------------------------------------------
// search_dft<HITS, VAR>: the search_mfma work decomposition (workgroup = 4 waves = 4 range
// blocks of one bucket, domain tiles staged through LDS, 4 tiles per double-buffered
// stage); per lane the chunk maximum of y over its 16 rows × the stage's tiles (all four
// transforms folded in).  Entries: [nwork*4][64] {float bits of max y (+inf = hit), tile}.
// VAR 1: exact path only (A/B of the guard).
// ---------------------------------------------------------------------------
__device__ inline floatx16_t mfma2(const half8_t& a0, const half8_t& b0, const half8_t& a1, const half8_t& b1,
                                   const floatx16_t& c)
{
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c, 0, 0, 0),
                                                  0, 0, 0);
}

constexpr int kDftChain = 1024;  // VAR bit: v_max3 chain for the row maximum

typedef float float2v_t __attribute__((ext_vector_type(2)));


// the five-MFMA form (kDft5): af = [s_b + u_b, s_b − u_b, γ, γ − δ, −δ − γ],
// bf = [s_a + u_a, s_a − u_a, 2(α + β), −2β, 2α]
template <bool PK = true>
__device__ inline float dft_tile_max5(const half8_t (&af)[5], const half8_t (&bf)[5], const floatx16_t& ny, float m)
{
    const floatx16_t z = {};
    const floatx16_t k1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bf[2], z, 0, 0, 0); // 2k1
    const floatx16_t p = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[0], z, 0, 0, 0);  // P = U + U'
    const floatx16_t q = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[1], z, 0, 0, 0);  // M = U − U'
    const floatx16_t pr = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bf[3], k1, 0, 0, 0); // 2Pr
    const floatx16_t pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], bf[4], k1, 0, 0, 0); // 2Pi
    float y[16];
    if constexpr (!PK) {
        // one row per instruction (A/B of the packed P ± M and fma below)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float X = p[i] + q[i], Xp = p[i] - q[i];
            y[i] = __builtin_fmaxf(X + __builtin_fabsf(pr[i]), Xp + __builtin_fabsf(pi[i])) + ny[i]; // h
        }
#pragma unroll
        for (int i = 0; i < 16; i += 2)
            m = __builtin_fmaxf(__builtin_fmaxf(m, y[i]), y[i + 1]);
        return m;
    }
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
        // two rows per packed instruction where no |·| modifier is needed
        const float2v_t P2 = {p[i], p[i + 1]}, M2 = {q[i], q[i + 1]};
        const float2v_t X = P2 + M2, Xp = P2 - M2; // 2U, 2U'
        const float2v_t t = {__builtin_fmaxf(X.x + __builtin_fabsf(pr[i]), Xp.x + __builtin_fabsf(pi[i])),
                             __builtin_fmaxf(X.y + __builtin_fabsf(pr[i + 1]), Xp.y + __builtin_fabsf(pi[i + 1]))};
        const float2v_t N2 = {ny[i], ny[i + 1]};
        const float2v_t yy = t + N2; // h = y/2
        y[i] = yy.x;
        y[i + 1] = yy.y;
    }
#pragma unroll
    for (int i = 0; i < 16; i += 2)
        m = __builtin_fmaxf(__builtin_fmaxf(m, y[i]), y[i + 1]);
    return m;
}

// the six-MFMA form (kDft6): af as dft_tile_max5, bf = [s_a + u_a, s_a − u_a, u_a − s_a, 2(α + β), −2β, 2α].
// The M GEMM accumulates onto P once with +(s_a − u_a) and once with −(s_a − u_a), giving 2U and 2U'
// in the MFMA (the five-MFMA form's two VALU per candidate for P ± M go away).  Exact in any
// accumulation order: with A0 = s_a + u_a, A2 = s_a − u_a (B0, B2 on the domain side),
// |A0| + |A2| = 2·max(|s_a|, |u_a|) ≤ 512 and |B0|, |B2| ≤ 2048, so every partial sum of P ± M is
// bounded by Σ_o (|A0·B0| + |A2·B2|) ≤ 16·2048·512 = 2^24.  Then the exact form's epilogue:
//   h = max(2U + |2Pr|, 2U' + |2Pi|) − Σb²/2   (ny = −Σb²/2; y = 2h).
__device__ inline float dft_tile_max6(const half8_t (&af)[5], const half8_t (&bf)[6], const floatx16_t& ny, float m)
{
    const floatx16_t z = {};
    const floatx16_t p = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[0], z, 0, 0, 0);  // P
    const floatx16_t k1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bf[3], z, 0, 0, 0); // 2k1
    const floatx16_t u = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[1], p, 0, 0, 0);  // P + M = 2U
    const floatx16_t pr = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bf[4], k1, 0, 0, 0); // 2Pr
    const floatx16_t v = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[2], p, 0, 0, 0);  // P − M = 2U'
    const floatx16_t pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], bf[5], k1, 0, 0, 0); // 2Pi
    float y[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        y[i] = __builtin_fmaxf(u[i] + __builtin_fabsf(pr[i]), v[i] + __builtin_fabsf(pi[i])) + ny[i];
#pragma unroll
    for (int i = 0; i < 16; i += 2)
        m = __builtin_fmaxf(__builtin_fmaxf(m, y[i]), y[i + 1]);
    return m;
}

// The guarded fast path (kDftFast6, exactness above kFast6Limit): P starts from C = −Σb²/2, so u' and
// v' carry the row constant and a candidate costs u' + |2Pr|, v' + |2Pi| and one step of a v_max3
// chain.  Only for tile pairs whose guard holds.
__device__ inline float dft_tile_max6_fast(const half8_t (&af)[5], const half8_t (&bf)[6], const floatx16_t& ny,
                                           float m)
{
    const floatx16_t z = {};
    const floatx16_t k1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bf[3], z, 0, 0, 0); // 2k1
    const floatx16_t p = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[0], ny, 0, 0, 0); // P − Σb²/2
    const floatx16_t pr = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bf[4], k1, 0, 0, 0); // 2Pr
    const floatx16_t u = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[1], p, 0, 0, 0);  // 2U − Σb²/2
    const floatx16_t pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], bf[5], k1, 0, 0, 0); // 2Pi
    const floatx16_t v = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[2], p, 0, 0, 0);  // 2U' − Σb²/2
#pragma unroll
    for (int i = 0; i < 16; ++i)
        m = __builtin_fmaxf(__builtin_fmaxf(m, u[i] + __builtin_fabsf(pr[i])), v[i] + __builtin_fabsf(pi[i]));
    return m;
}

// The six-MFMA form for two range blocks sharing one domain tile (search_dft2<…, true>): the tile's
// A fragments and row constants are read once for both blocks.
__device__ inline void dft_tile_max6x2(const half8_t (&af)[5], const half8_t (&ba)[6], const half8_t (&bb)[6],
                                       const floatx16_t& ny, float& ma, float& mb)
{
    const floatx16_t z = {};
    const floatx16_t pa = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], ba[0], z, 0, 0, 0);
    const floatx16_t pb = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bb[0], z, 0, 0, 0);
    const floatx16_t ka = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], ba[3], z, 0, 0, 0);
    const floatx16_t kb = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bb[3], z, 0, 0, 0);
    const floatx16_t ua = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], ba[1], pa, 0, 0, 0);
    const floatx16_t ub = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bb[1], pb, 0, 0, 0);
    const floatx16_t ra = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], ba[4], ka, 0, 0, 0);
    const floatx16_t rb = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bb[4], kb, 0, 0, 0);
    const floatx16_t va = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], ba[2], pa, 0, 0, 0);
    const floatx16_t vb = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bb[2], pb, 0, 0, 0);
    const floatx16_t ia = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], ba[5], ka, 0, 0, 0);
    const floatx16_t ib = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], bb[5], kb, 0, 0, 0);
    float ya[16], yb[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { // h = y/2 (ny = −Σb²/2)
        ya[i] = __builtin_fmaxf(ua[i] + __builtin_fabsf(ra[i]), va[i] + __builtin_fabsf(ia[i])) + ny[i];
        yb[i] = __builtin_fmaxf(ub[i] + __builtin_fabsf(rb[i]), vb[i] + __builtin_fabsf(ib[i])) + ny[i];
    }
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
        ma = __builtin_fmaxf(__builtin_fmaxf(ma, ya[i]), ya[i + 1]);
        mb = __builtin_fmaxf(__builtin_fmaxf(mb, yb[i]), yb[i + 1]);
    }
}

template <int VAR>
__device__ inline float dft_tile_max4(const half8_t (&af)[4], const half8_t (&bf)[kDftRangeFrags],
                                      const floatx16_t& ny, bool fast, float m)
{
    const floatx16_t z = {};
    // af: [s_b, u_b, γ, δ];  bf: [s_a, u_a, 4s_a, 4u_a, α, β, −α]
    if constexpr ((VAR & 16) != 0) {
        // ABLATION (tuning only, wrong results): the exact epilogue on fake accumulators
        floatx16_t u, v, pr, pi;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float b = __builtin_bit_cast(float, __builtin_bit_cast(uint4, af[i & 3]).x);
            u[i] = b + (float)i;
            v[i] = b - (float)i;
            pr[i] = b * 0.5f;
            pi[i] = ny[i];
        }
        float m2 = m;
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            const float y0 = __builtin_fmaf(
                __builtin_fmaxf(u[i] + __builtin_fabsf(pr[i]), v[i] + __builtin_fabsf(pi[i])), 4.0f, ny[i]);
            const float y1 = __builtin_fmaf(__builtin_fmaxf(u[i + 1] + __builtin_fabsf(pr[i + 1]),
                                                            v[i + 1] + __builtin_fabsf(pi[i + 1])),
                                            4.0f, ny[i + 1]);
            m2 = __builtin_fmaxf(m2, __builtin_fmaxf(y0, y1));
        }
        (void)bf;
        (void)fast;
        return m2;
    }
    const floatx16_t pr = mfma2(af[2], bf[4], af[3], bf[5], z);
    float m0 = m, m1 = -__builtin_inff();
    if ((VAR & 1) == 0 && fast) {
        const floatx16_t pi = mfma2(af[2], bf[5], af[3], bf[6], z);
        const floatx16_t u = mfma2(af[0], bf[2], af[1], bf[3], ny);  // 4U − Σb²
        const floatx16_t v = mfma2(af[0], bf[3], af[1], bf[2], ny);  // 4U' − Σb²
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            m0 = __builtin_fmaxf(m0, __builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(pr[i]), 4.0f, u[i]),
                                                     __builtin_fmaf(__builtin_fabsf(pi[i]), 4.0f, v[i])));
            m1 = __builtin_fmaxf(m1, __builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(pr[i + 1]), 4.0f, u[i + 1]),
                                                     __builtin_fmaf(__builtin_fabsf(pi[i + 1]), 4.0f, v[i + 1])));
        }
    } else if constexpr ((VAR & 8) != 0) {
        // ABLATION (tuning only, wrong results): MFMAs with a one-value epilogue
        const floatx16_t pi = mfma2(af[2], bf[5], af[3], bf[6], z);
        const floatx16_t u = mfma2(af[0], bf[0], af[1], bf[1], z);
        const floatx16_t v = mfma2(af[0], bf[1], af[1], bf[0], z);
        m0 = __builtin_fmaxf(m0, u[0] + v[0] + pr[0] + pi[0] + ny[0]);
    } else if constexpr ((VAR & kDftChain) != 0) {
        // the row maximum as one v_max3 chain over the 16 candidates (8 instead of the 12 the
        // pairwise tree below compiles to): 76 instead of 80 VALU per tile pair in the loop,
        // −1.3 % search time in a 20-round interleaved A/B (tools/ab_mfma.py d,dc)
        const floatx16_t u = mfma2(af[0], bf[0], af[1], bf[1], z);   // U
        const floatx16_t v = mfma2(af[0], bf[1], af[1], bf[0], z);   // U'
        const floatx16_t pi = mfma2(af[2], bf[5], af[3], bf[6], z);  // Pi
        float y[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
            y[i] = __builtin_fmaf(__builtin_fmaxf(u[i] + __builtin_fabsf(pr[i]), v[i] + __builtin_fabsf(pi[i])), 4.0f,
                                  ny[i]);
#pragma unroll
        for (int i = 0; i < 16; i += 2)
            m0 = __builtin_fmaxf(__builtin_fmaxf(m0, y[i]), y[i + 1]);
        return m0;
    } else {
        const floatx16_t u = mfma2(af[0], bf[0], af[1], bf[1], z);   // U
        const floatx16_t v = mfma2(af[0], bf[1], af[1], bf[0], z);   // U'
        const floatx16_t pi = mfma2(af[2], bf[5], af[3], bf[6], z);  // Pi
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            const float y0 = __builtin_fmaf(
                __builtin_fmaxf(u[i] + __builtin_fabsf(pr[i]), v[i] + __builtin_fabsf(pi[i])), 4.0f, ny[i]);
            const float y1 = __builtin_fmaf(
                __builtin_fmaxf(u[i + 1] + __builtin_fabsf(pr[i + 1]), v[i + 1] + __builtin_fabsf(pi[i + 1])), 4.0f,
                ny[i + 1]);
            m0 = __builtin_fmaxf(m0, __builtin_fmaxf(y0, y1));
        }
    }
    return __builtin_fmaxf(m0, m1);
}

template <int VAR>
__device__ inline float dft_tile_max(const half8_t (&af)[DftForm<VAR>::KS], const half8_t (&bf)[DftForm<VAR>::NBF],
                                     const floatx16_t& ny, bool fast, float m)
{
    if constexpr (DftForm<VAR>::F5) {
        static_assert((VAR & 1) != 0, "the five-MFMA form has no guarded fast path");
        (void)fast;
        return dft_tile_max5<(VAR & kDftScalar) == 0>(af, bf, ny, m);
    } else if constexpr (DftForm<VAR>::F6) {
        static_assert((VAR & 1) != 0, "the six-MFMA form's guarded path is kDftFast6");
        if constexpr (DftForm<VAR>::FAST6) {
            if (fast)
                return dft_tile_max6_fast(af, bf, ny, m);
        }
        (void)fast;
        return dft_tile_max6(af, bf, ny, m);
    } else {
        return dft_tile_max4<VAR>(af, bf, ny, fast, m);
    }
}

// MASK (CHUNKED search): masks[0] gets the chunk tiles attaining the lane's maximum, masks[1]
// (HITS) the tiles holding a hit (y ≥ hl), bit k for tile q0 + k
__device__ inline floatx16_t lds_row_consts(const uint4* p)
{
    floatx16_t r;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
        const uint4 v = p[c4];
        r[4 * c4 + 0] = __uint_as_float(v.x);
        r[4 * c4 + 1] = __uint_as_float(v.y);
        r[4 * c4 + 2] = __uint_as_float(v.z);
        r[4 * c4 + 3] = __uint_as_float(v.w);
    }
    return r;
}

// One tile pair of the six-MFMA form with the guarded fast path (kDftFast6).  Both paths issue
// the same six MFMAs; only P's C operand differs — the tile's −Σb²/2 row constants when the guard
// holds, the stage's zero block when it does not (a wave-uniform choice of address, so one MFMA
// sequence and one register allocation serve both) — and the epilogue: the folded form
// (2 VALU + one v_max3 step per candidate), or the exact one with the constants read after the
// MFMAs.  lc: the tile's row constants ([2][16] lane-half layout), h: the lane half.
template <int ABL = 0>
__device__ inline float dft_tile_max6g(const half8_t (&af)[5], const half8_t (&bf)[6], const uint4* la, uint32_t ic,
                                       uint32_t iz, uint32_t h, bool fast, float m)
{
    if constexpr (ABL == 16) {
        // ABLATION (tuning only, wrong results): the fast epilogue on the fragments' bits, no MFMA
        const floatx16_t c = lds_row_consts(la + (fast ? ic : iz) + h * 4);
        auto bits = [&](const half8_t& x, int i) { return __builtin_bit_cast(uint4, x)[i & 3]; };
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float u = c[i] + __uint_as_float(bits(af[i >> 2], i)), pr = __uint_as_float(bits(bf[i >> 2], i));
            const float v = __uint_as_float(bits(af[(i >> 2) + 1], i)), pi = __uint_as_float(bits(bf[(i >> 2) + 2], i));
            m = __builtin_fmaxf(__builtin_fmaxf(m, u + __builtin_fabsf(pr)), v + __builtin_fabsf(pi));
        }
        return m;
    }
    // one base pointer, a selected index: the compiler keeps the read's underlying LDS object and
    // does not wait for the other stage buffer's pending LDS-DMA (a selected pointer made it)
    const uint4* lc = la + ic;
    const floatx16_t c = lds_row_consts(la + (fast ? ic : iz) + h * 4);
    const floatx16_t z = {};
    const floatx16_t k1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bf[3], z, 0, 0, 0); // 2k1
    const floatx16_t p = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[0], c, 0, 0, 0);  // P (− Σb²/2)
    const floatx16_t pr = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bf[4], k1, 0, 0, 0); // 2Pr
    const floatx16_t u = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[1], p, 0, 0, 0);  // 2U (− Σb²/2)
    const floatx16_t pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], bf[5], k1, 0, 0, 0); // 2Pi
    const floatx16_t v = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[2], p, 0, 0, 0);  // 2U' (− Σb²/2)
    if constexpr (ABL == 8) // ABLATION (tuning only, wrong results): the MFMAs with a one-value epilogue
        return __builtin_fmaxf(m, (u[0] + pr[0]) + (v[0] + pi[0]));
    if (fast) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            m = __builtin_fmaxf(__builtin_fmaxf(m, u[i] + __builtin_fabsf(pr[i])), v[i] + __builtin_fabsf(pi[i]));
        return m;
    }
    const floatx16_t ny = lds_row_consts(lc + h * 4);
    float y[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        y[i] = __builtin_fmaxf(u[i] + __builtin_fabsf(pr[i]), v[i] + __builtin_fabsf(pi[i])) + ny[i];
#pragma unroll
    for (int i = 0; i < 16; i += 2)
        m = __builtin_fmaxf(__builtin_fmaxf(m, y[i]), y[i + 1]);
    return m;
}

// kDftFast6 guard bits of a 4-tile chunk: bit k set iff the block's R6 ≤ tile t0 + k's threshold
// (one scalar load of four thresholds; trmax is padded by 4 entries), masked to the chunk's ne tiles
__device__ inline uint32_t dft_guard_bits(const int32_t* __restrict__ trmax, uint32_t t0, uint32_t ne, uint32_t r1)
{
    t0 = __builtin_amdgcn_readfirstlane(t0);
    const __attribute__((address_space(4))) int32_t* rp =
        (const __attribute__((address_space(4))) int32_t*)(uintptr_t)(trmax + t0);
    const int32_t g0 = rp[0], g1 = rp[1], g2 = rp[2], g3 = rp[3], ri = (int32_t)r1;
    const uint32_t g = ((ri <= g0) ? 1u : 0u) | ((ri <= g1) ? 2u : 0u) | ((ri <= g2) ? 4u : 0u) | ((ri <= g3) ? 8u : 0u);
    return g & ((1u << ne) - 1u);
}

template <int VAR, bool MASK = false, bool HITS = false>
__device__ inline float dft_compute_stage(const uint4* __restrict__ la, uint32_t nt, uint32_t lane,
                                          const half8_t (&bf)[DftForm<VAR>::NBF], uint32_t tb,
                                          const uint2* __restrict__ tguard, uint32_t r1, uint32_t q0 = 0,
                                          uint32_t q1 = ~0u, uint32_t* masks = nullptr, float hl = 0.0f,
                                          uint32_t iz = 0, const int32_t* __restrict__ trmax = nullptr)
{
    constexpr int KS = DftForm<VAR>::KS;
    const uint4* lc = la + nt * (uint32_t)KS * 64u;
    const uint32_t h = lane >> 5;
    float cm = -__builtin_inff();
    // the chunk's fast-path guards, loaded up front (wave-uniform scalar loads)
    uint32_t gfast = 0;
    // the tile index is wave-uniform: readfirstlane + the constant address space make the guard
    // loads scalar, which the vmcnt waits of the stage's LDS-DMA do not serialise with
    const uint32_t t0 = __builtin_amdgcn_readfirstlane(tb + q0), ne = __builtin_amdgcn_readfirstlane(min(q1, nt) - q0);
    if constexpr (DftForm<VAR>::FAST6) {
        gfast = dft_guard_bits(trmax, t0, ne, r1);
    } else if constexpr ((VAR & 1) == 0) {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (k < ne) {
                const __attribute__((address_space(4))) uint32_t* gp =
                    (const __attribute__((address_space(4))) uint32_t*)(uintptr_t)(tguard + t0 + k);
                gfast |= ((uint64_t)r1 * gp[0] + gp[1] <= (uint64_t)kExactLimit) ? (1u << k) : 0u;
            }
    }
    auto tile = [&](uint32_t q) {
        // ABLATION bit 32 (tuning only, wrong results): every tile reuses tile 0's operands
        const uint32_t qq = (VAR & 32) ? 0u : q;
        half8_t af[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s)
            af[s] = __builtin_bit_cast(half8_t, la[(qq * KS + s) * 64 + lane]);
        if constexpr (DftForm<VAR>::FAST6) {
            const bool fast = (gfast >> (q - q0)) & 1u;
            const uint32_t ic = nt * (uint32_t)KS * 64u + qq * kDftCS;
            if constexpr (MASK) { // TMASK: the tile's own maximum first, then the chunk's tiles attaining it
                const float tm = dft_tile_max6g<VAR & (8 | 16)>(af, bf, la, ic, iz, h, fast, -__builtin_inff());
                const uint32_t bit = 1u << (q - q0);
                masks[0] = tm > cm ? bit : (tm == cm ? masks[0] | bit : masks[0]);
                if constexpr (HITS)
                    masks[1] |= tm >= hl ? bit : 0u;
                cm = __builtin_fmaxf(cm, tm);
            } else {
                cm = dft_tile_max6g<VAR & (8 | 16)>(af, bf, la, ic, iz, h, fast, cm);
            }
            return;
        }
        floatx16_t ny;
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
            const uint4 v = lc[qq * kDftCS + h * 4 + c4];
            ny[4 * c4 + 0] = __uint_as_float(v.x);
            ny[4 * c4 + 1] = __uint_as_float(v.y);
            ny[4 * c4 + 2] = __uint_as_float(v.z);
            ny[4 * c4 + 3] = __uint_as_float(v.w);
        }
        // wave-uniform guard: every partial sum of 4U − Σb² stays within 2^24
        const bool fast = (gfast >> (q - q0)) & 1u;
        if constexpr (MASK) {
            const float tm = dft_tile_max<VAR>(af, bf, ny, fast, -__builtin_inff());
            const uint32_t bit = 1u << (q - q0);
            masks[0] = tm > cm ? bit : (tm == cm ? masks[0] | bit : masks[0]);
            if constexpr (HITS)
                masks[1] |= tm >= hl ? bit : 0u;
            cm = __builtin_fmaxf(cm, tm);
        } else {
            cm = dft_tile_max<VAR>(af, bf, ny, fast, cm);
        }
    };
    const uint32_t qe = min(q1, nt);
    if constexpr ((VAR & kDftUnroll) != 0) {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (q0 + k < qe)
                tile(q0 + k);
    } else {
        for (uint32_t q = q0; q < qe; ++q)
            tile(q);
    }
    return cm;
}

// stage_tiles by buffer_load … lds in whole-wave pieces (1 KiB each): the stage's nt·KS A-fragment
// pieces and its one constants piece (kDftCS = 16 uint4 per tile: 4 tiles are one piece; a shorter
// last stage reads the next tiles' constants or the allocation's 1 KiB of slack, never used).  The
// loop, the LDS destination (M0) and the source offset (soffset) are wave-uniform: every piece costs
// scalar instructions only, the lane's voffset (lane·16) is fixed.
template <int KS, uint32_t WAVES>
__device__ inline void stage_tiles_buf(uint4* dst, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rc, uint32_t tb,
                                       uint32_t nt)
{
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t voff = (threadIdx.x & 63u) * 16u;
    const uint32_t tbu = __builtin_amdgcn_readfirstlane(tb), npa = __builtin_amdgcn_readfirstlane(nt * (uint32_t)KS);
    for (uint32_t p = wv; p <= npa; p += WAVES) {
        auto* l = (__attribute__((address_space(3))) void*)(dst + p * 64u);
        if (p < npa)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, l, 16, voff, (tbu * (uint32_t)KS + p) * 1024u, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, l, 16, voff, tbu * kDftCS * 16u, 0, 0);
    }
}

constexpr uint32_t kDftBlocksPerWG = 8; // waves (range blocks) sharing one LDS domain stage

// CHUNKED (the SEA engine's tiled form, fracenc_tp.hip): tiles are in ΣD4 order, not domain
// order, so instead of the first chunk attaining each lane's maximum every chunk's maximum is
// written, entry ((choff[work] + chunk)·WAVES + wave)·64 + lane, and resolve_dft keeps all ties.
// TMASK (not CHUNKED, slotbest): each lane also tracks which tiles of its best chunk attain its maximum (or
// hold a hit), and the slot word carries them, so resolve_dft re-evaluates those tiles instead of the whole
// chunk.  Costs the tile-pair epilogue a compare per tile: chosen where the resolve, not the search, dominates.
template <bool HITS, int VAR, uint32_t WAVES = 4, uint32_t TPS = kTilesPerStage, bool CHUNKED = false,
          bool TMASK = false>
__global__ void __launch_bounds__(64 * WAVES) search_dft(DftArgs d)
{
    static_assert(kTuningBuild || (VAR & (8 | 16 | 32 | 64 | 256 | 512)) == 0,
                  "search_dft ablations exist only in FRAC_TUNING builds");
    static_assert(!(TMASK && CHUNKED), "CHUNKED entries carry their own tile masks");
    if (past_plan(d.m))
        return;
    const MfmaSearchArgs& a = d.m;
    constexpr int KS = DftForm<VAR>::KS, NBF = DftForm<VAR>::NBF;
    constexpr uint32_t kTilesPerStage = TPS; // LDS stage; chunks stay 4 tiles (resolve_dft)
    constexpr int STAGE = kTilesPerStage * KS * 64 + kTilesPerStage * kDftCS;
    // kDftFast6: each stage buffer ends in 8 zero uint4, the row constants of a tile pair that runs
    // the exact epilogue (written here, published by the first stage barrier, never a DMA target).
    // Inside the stage's own array, so the compiler still tells these reads from the other
    // buffer's pending LDS-DMA (a separate array made it wait vmcnt(0) before every tile)
    constexpr int ZTAIL = DftForm<VAR>::FAST6 ? 8 : 0;
    __shared__ uint4 lds0[STAGE + ZTAIL];
    __shared__ uint4 lds1[STAGE + ZTAIL];
    if constexpr (DftForm<VAR>::FAST6)
        if (threadIdx.x < 2 * ZTAIL)
            (threadIdx.x < ZTAIL ? lds0 : lds1)[STAGE + (threadIdx.x % ZTAIL)] = make_uint4(0u, 0u, 0u, 0u);
    const uint4 wk = a.work[blockIdx.x];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const bool active = wv < wk.y;
    const uint32_t blk = wk.x + (active ? wv : 0u);
    const uint32_t r1 = __builtin_amdgcn_readfirstlane(d.rguard[blk]);

    half8_t bf[NBF];
#pragma unroll
    for (int f = 0; f < NBF; ++f)
        bf[f] = __builtin_bit_cast(half8_t, a.rfrags[((size_t)blk * NBF + f) * 64 + lane]);
    float hl = 0.0f;
    if constexpr (HITS) { // S16 ≤ H  ⇔  y ≥ 16Σa² − H  (exact integers below 2^24; halved exactly for h)
        hl = (float)((int32_t)a.rconst[blk * 32 + (lane & 31u)] - (int32_t)a.hitH);
        if constexpr (DftForm<VAR>::HALF)
            hl *= 0.5f;
    }
    // the forms that track h = y/2 store y = 2h (exact) in the entries
    constexpr float kOut = DftForm<VAR>::HALF ? 2.0f : 1.0f;

    float best = -__builtin_inff();
    uint32_t btile = 0, bmask = 0xfu;
    uint32_t masks[2] = {0u, 0u};
    auto finish_stage = [&](float cm, uint32_t tb) {
        if constexpr (CHUNKED) {
            static_assert(TPS == 4, "chunk entries assume 4-tile stages");
            // the entry carries the chunk's tile mask in bits 28..31 of its tile (resolve_dft<true>
            // evaluates only those tiles): the hit tiles when the chunk holds a hit, else the
            // tiles attaining the maximum
            uint32_t msk = masks[0];
            if constexpr (HITS)
                if (cm >= hl) {
                    cm = __builtin_inff();
                    msk = masks[1];
                }
            if (active)
                a.entries[((size_t)(d.choff[blockIdx.x] + (tb - wk.z) / 4u) * WAVES + wv) * 64 + lane] =
                    make_uint2(__float_as_uint(cm * kOut), tb | (msk << 28));
            masks[0] = masks[1] = 0u;
            return;
        }
        // any hit in the chunk: the first-hit chunk wins. (A per-tile mask here, as the CHUNKED
        // entries carry, cost 4% of this kernel in a 30-sample A/B for 0.1 ms less resolve: only TMASK.)
        uint32_t msk = 0xfu;
        if constexpr (TMASK) {
            msk = masks[0];
            if constexpr (HITS)
                msk = cm >= hl ? masks[1] : msk;
            masks[0] = masks[1] = 0u;
        }
        if constexpr (HITS)
            cm = cm >= hl ? __builtin_inff() : cm;
        if (cm > best) {
            best = cm;
            btile = tb;
            bmask = msk;
        }
    };
    const uint32_t nstage = (wk.w - wk.z + kTilesPerStage - 1) / kTilesPerStage;
    auto stage_nt = [&](uint32_t st) { return min((uint32_t)kTilesPerStage, wk.w - (wk.z + st * kTilesPerStage)); };
    // ABLATION bits (tuning only, wrong results): 64 no LDS-DMA and no barrier after the first
    // stages; 256 no LDS-DMA (barriers kept); 512 no barrier (LDS-DMA kept)
    constexpr bool NODMA = (VAR & 64) != 0;
    constexpr bool SKIPDMA = NODMA || (VAR & 256) != 0, SKIPBAR = NODMA || (VAR & 512) != 0;
    auto stage = [&](uint4* dst, uint32_t tb, uint32_t nt) {
        if constexpr ((VAR & kDftBufDma) != 0) // raw buffers (no range check: the pieces are in bounds)
            stage_tiles_buf<KS, WAVES>(
                dst, __builtin_amdgcn_make_buffer_rsrc((void*)a.dtiles, 0, 0xffffffffu, 0x00020000),
                __builtin_amdgcn_make_buffer_rsrc((void*)a.dconst, 0, 0xffffffffu, 0x00020000), tb, nt);
        else
            stage_tiles<KS, 64 * WAVES, kDftCS>(dst, a.dtiles, a.dconst, tb, nt);
    };
    if constexpr ((VAR & kDftPrio) != 0)
        if (wv >= WAVES / 2)
            __builtin_amdgcn_s_setprio(1);
#ifdef FRAC_CLOCK_STAMP
    // diagnostic build only (tools/clock_stamp.py, MI355X_MICROARCH.md "DVFS give-back"): the shader
    // clock over this workgroup's loop is Δs_memtime ÷ Δs_memrealtime × 100 MHz
    const unsigned long long ck0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    if (nstage)
        stage(lds0, wk.z, stage_nt(0));
    for (uint32_t st = 0; st < nstage; st += 2) {
        {
            const uint32_t tb = wk.z + st * kTilesPerStage;
            if (!SKIPBAR || st < 2)
                stage_barrier();
            if (st + 1 < nstage && (!SKIPDMA || st == 0))
                stage(lds1, tb + kTilesPerStage, stage_nt(st + 1));
            for (uint32_t c0 = 0; c0 < stage_nt(st); c0 += 4)
                finish_stage(dft_compute_stage<VAR, CHUNKED || TMASK, HITS>(lds0, stage_nt(st), lane, bf, tb, d.tguard, r1, c0,
                                                                   c0 + 4, masks, hl, STAGE, d.trmax),
                             tb + c0);
        }
        if (st + 1 < nstage) {
            const uint32_t tb = wk.z + (st + 1) * kTilesPerStage;
            if (!SKIPBAR || st < 2)
                stage_barrier();
            if (st + 2 < nstage && !SKIPDMA)
                stage(lds0, tb + kTilesPerStage, stage_nt(st + 2));
            for (uint32_t c0 = 0; c0 < stage_nt(st + 1); c0 += 4)
                finish_stage(dft_compute_stage<VAR, CHUNKED || TMASK, HITS>(lds1, stage_nt(st + 1), lane, bf, tb, d.tguard, r1,
                                                                   c0, c0 + 4, masks, hl, STAGE, d.trmax),
                             tb + c0);
        }
    }
#ifdef FRAC_CLOCK_STAMP
    {
        const unsigned long long ck1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
        // where the workgroup ran: HW_ID (CU, SE, …) and XCC_ID, read by s_getreg (hwreg 4 and 20)
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        if (threadIdx.x == 0 && d.stamps) { // vector stores from lane 0; nothing in the kernel reads them
            ulonglong2* sp = reinterpret_cast<ulonglong2*>(d.stamps + (size_t)blockIdx.x * kClockStampWords);
            sp[0] = make_ulonglong2(ck0, ck1);
            sp[1] = make_ulonglong2(rt0, rt1);
            sp[2] = make_ulonglong2((unsigned long long)hw | ((unsigned long long)xcc << 32),
                                    (unsigned long long)wk.z | ((unsigned long long)wk.w << 32));
        }
    }
#endif
    if (active && !CHUNKED) {
        if (d.slotbest) {
            // lanes l and l + 32 hold one range slot's two row halves: the greater y, among equal y the earlier
            // chunk, and which halves attain it there (both: resolve_dft evaluates both halves' rows)
            const uint32_t y0 = fmap(best * kOut), t0 = btile;
            const uint32_t y1 = (uint32_t)__shfl_xor((int)y0, 32, 64), t1 = (uint32_t)__shfl_xor((int)t0, 32, 64);
            const uint32_t m1 = TMASK ? (uint32_t)__shfl_xor((int)bmask, 32, 64) : 0xfu;
            const bool first = lane < 32u;
            const uint32_t ym = first ? y0 : y1, tm = first ? t0 : t1; // this half (lane < 32: half 0)
            const uint32_t yo = first ? y1 : y0, to = first ? t1 : t0; // the other half
            if (first) {
                uint32_t tile = tm, hm = 1u, mk = bmask;
                if (yo > ym || (yo == ym && to < tm)) {
                    tile = to;
                    hm = 2u;
                    mk = m1;
                } else if (yo == ym && to == tm) {
                    hm = 3u;
                    mk |= m1; // both halves' rows are evaluated on every tile of the union
                }
                const unsigned long long w = ((unsigned long long)max(ym, yo) << 32) |
                                             ((kSlotBestTileMax - tile) << 6) | (mk << 2) | hm;
                atomicMax(d.slotbest + (size_t)blk * 32 + lane, w);
            }
        } else {
            a.entries[(size_t)(blockIdx.x * WAVES + wv) * 64 + lane] = make_uint2(__float_as_uint(best * kOut), btile);
        }
    }
}

// ---------------------------------------------------------------------------
// search_dft2<HITS>: the exact form with two range blocks per wave (4-wave workgroups, 8 blocks
// per workgroup, the entry layout of search_dft<…, 8>): a tile's A fragments and −Σb² row
// constants are read from LDS once for both blocks, half the LDS bytes per (block, tile) pair.
// 3 waves per SIMD (3 workgroups per CU) instead of 4.
// ---------------------------------------------------------------------------
// F6: the six-MFMA form (dft_tile_max6x2), 2 waves per SIMD
template <bool HITS, bool F6 = false>
__global__ void __launch_bounds__(256, F6 ? 2 : 3) search_dft2(DftArgs d)
{
    const MfmaSearchArgs& a = d.m;
    constexpr int VAR = 1 | kDftChain | (F6 ? kDft6 : 0);
    constexpr int KS = DftForm<VAR>::KS, NBF = DftForm<VAR>::NBF;
    constexpr int STAGE = kTilesPerStage * KS * 64 + kTilesPerStage * kDftCS;
    __shared__ uint4 lds0[STAGE];
    __shared__ uint4 lds1[STAGE];
    const uint4 wk = a.work[blockIdx.x];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    bool act[2];
    half8_t bf[2][NBF];
    float hl[2] = {0.0f, 0.0f}, best[2];
    uint32_t btile[2] = {0u, 0u};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t b = 2 * wv + k;
        act[k] = b < wk.y;
        const uint32_t blk = wk.x + (act[k] ? b : 0u);
#pragma unroll
        for (int f = 0; f < NBF; ++f)
            bf[k][f] = __builtin_bit_cast(half8_t, a.rfrags[((size_t)blk * NBF + f) * 64 + lane]);
        if constexpr (HITS)
            hl[k] = (float)((int32_t)a.rconst[blk * 32 + (lane & 31u)] - (int32_t)a.hitH) * (F6 ? 0.5f : 1.0f);
        best[k] = -__builtin_inff();
    }
    const uint32_t h = lane >> 5;
    auto compute = [&](const uint4* la, uint32_t nt, uint32_t tb) {
        const uint4* lc = la + nt * (uint32_t)KS * 64u;
        float cm[2] = {-__builtin_inff(), -__builtin_inff()};
        for (uint32_t q = 0; q < nt; ++q) {
            half8_t af[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s)
                af[s] = __builtin_bit_cast(half8_t, la[(q * KS + s) * 64 + lane]);
            floatx16_t ny;
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
                const uint4 v = lc[q * kDftCS + h * 4 + c4];
                ny[4 * c4 + 0] = __uint_as_float(v.x);
                ny[4 * c4 + 1] = __uint_as_float(v.y);
                ny[4 * c4 + 2] = __uint_as_float(v.z);
                ny[4 * c4 + 3] = __uint_as_float(v.w);
            }
            if constexpr (F6) {
                dft_tile_max6x2(af, bf[0], bf[1], ny, cm[0], cm[1]);
            } else {
#pragma unroll
                for (int k = 0; k < 2; ++k)
                    cm[k] = dft_tile_max<VAR>(af, bf[k], ny, false, cm[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            float c = cm[k];
            if constexpr (HITS) // any hit in the chunk: the first-hit chunk wins
                c = c >= hl[k] ? __builtin_inff() : c;
            if (c > best[k]) {
                best[k] = c;
                btile[k] = tb;
            }
        }
    };
    const uint32_t nstage = (wk.w - wk.z + kTilesPerStage - 1) / kTilesPerStage;
    auto stage_nt = [&](uint32_t st) { return min((uint32_t)kTilesPerStage, wk.w - (wk.z + st * kTilesPerStage)); };
    if (nstage)
        stage_tiles<KS, 256, kDftCS>(lds0, a.dtiles, a.dconst, wk.z, stage_nt(0));
    for (uint32_t st = 0; st < nstage; st += 2) {
        {
            const uint32_t tb = wk.z + st * kTilesPerStage;
            stage_barrier();
            if (st + 1 < nstage)
                stage_tiles<KS, 256, kDftCS>(lds1, a.dtiles, a.dconst, tb + kTilesPerStage, stage_nt(st + 1));
            compute(lds0, stage_nt(st), tb);
        }
        if (st + 1 < nstage) {
            const uint32_t tb = wk.z + (st + 1) * kTilesPerStage;
            stage_barrier();
            if (st + 2 < nstage)
                stage_tiles<KS, 256, kDftCS>(lds0, a.dtiles, a.dconst, tb + kTilesPerStage, stage_nt(st + 2));
            compute(lds1, stage_nt(st + 1), tb);
        }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (act[k])
            a.entries[(size_t)(blockIdx.x * kDftBlocksPerWG + 2 * wv + k) * 64 + lane] =
                make_uint2(__float_as_uint(best[k] * (F6 ? 2.0f : 1.0f)), btile[k]); // F6 tracks h = y/2
}

// ---------------------------------------------------------------------------
// resolve_dft: one wave per range (resolve_mfma's lane map: tile row i = l>>2, pixel
// slice g = l&3).  The greatest entry y over the block's splits and lane halves gives the
// target error S16 = 16Σa² − y (exact regime) or flags the range for the fp32 fallback;
// the chunk(s) holding it are re-evaluated with exact integers for all four transforms,
// keeping the least selection key (first hit in (domain, transform) order, else least
// error with ties to the earliest domain, then the later transform).
// ---------------------------------------------------------------------------
// SORTED (tiles in ΣD4 order, fracenc_tp.hip): rows and tiles are not in domain order, so the
// least key over every matching row of every tile of the chunk is taken (no first-row shortcut).
// One slot's least key and the winner's sums (bestk = kKeyNone: padding slot, or no eligible domain).
// FLIP: the slot holds a T = 8 range's flipped copy (dft_range_prep flip_from), whose rotation t' is the
// reference's transform 4 + (−t' mod 4); the keys carry the reference's transform and a.T.
struct DftResolved {
    unsigned long long bestk = kKeyNone;
    uint32_t bx = 0, bs1 = 0, bs2 = 0, sr1 = 0, sr2 = 0;
};

template <bool SORTED>
__device__ inline DftResolved resolve_dft_eval(const MfmaResolveArgs& a, uint32_t slot, int lane, bool flip)
{
    constexpr int PG = 16, T = 4; // T: the rotations evaluated per slot
    const uint32_t TK = a.T;      // the transforms of the keys (4, or 8 with the flipped copies)
    DftResolved res;
    const int ri = a.slot_range[slot];
    // the slot-only loads go out with the padding check's (slot < nslots: in bounds either way)
    const unsigned long long sb = a.slotbest ? a.slotbest[slot] : 0ull;
    const int64_t sa16 = (int64_t)a.rconst[slot];
    const int i = lane >> 2, g = lane & 3;
    const uint4* rp4 = reinterpret_cast<const uint4*>(a.rorb + (size_t)slot * 32 + g * (PG / 2));
    const uint4 r0 = rp4[0], r1 = rp4[1];
    if (ri < 0)
        return res;
    const uint32_t blk = slot >> 5, col = slot & 31u;
    // lane (i, g) holds orbits 4g..4g+3 of the range as pixel pairs (dft_range_prep) and meets
    // the same orbits of a domain row (tile-order pool, dft_domain_build). With fwd(t) = g^t,
    //   X_t = Σ_q r(q)·D4(fwd_t q) = Σ_{o,k} r_{o,k}·D_{o,k+t}:
    // t = 0 pairs (A, B) = (D0|D1, D2|D3), t = 2 the swapped pairs (B, A), t = 1 the rotated
    // pairs (D1|D2, D3|D0) = (alignbit(B, A, 16), alignbit(A, B, 16)) and t = 3 those swapped —
    // two v_alignbit per orbit for all four transforms.
    const uint32_t rp[PG / 2] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    constexpr uint32_t kOnes = 0x00010001u;
    uint32_t sr2u = 0, sr1 = 0;
#pragma unroll
    for (int q = 0; q < PG / 2; ++q) {
        sr2u = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, rp[q]), __builtin_bit_cast(ushort2_t, rp[q]), sr2u,
                                      false);
        sr1 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, rp[q]), __builtin_bit_cast(ushort2_t, kOnes), sr1,
                                     false);
    }
    // every quad holds the whole range: the sums are wave-uniform (scalar registers from here on)
    sr2u = (uint32_t)__builtin_amdgcn_readfirstlane((int)quad_sum(sr2u));
    sr1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)quad_sum(sr1));
    const int sr2 = (int)sr2u; // Σr² ≤ 64·255²
    // the greatest entry y (vmax) over the block's splits and lane halves, and the chunk(s) holding it
    unsigned long long bestk = kKeyNone;
    uint32_t bx = 0, bs1 = 0, bs2 = 0; // X_t, ΣD4, ΣD4² of bestk's candidate (fit_rstat)
    float vmax = -__builtin_inff();
    bool exact = false, hit = false;
    int64_t target = -1;
    auto set_target = [&]() {
        const bool sentinel = vmax == __builtin_inff();
        exact = sentinel || vmax > (float)(sa16 - kExactLimit);
        target = exact && !sentinel ? sa16 - (int64_t)vmax : -1;
        hit = a.hitH >= 0 && (sentinel || (target >= 0 && target <= a.hitH));
    };
    // re-evaluate chunk `tile0` (4 tiles from there; SORTED: the tiles in tmask) on the rows of lane half h,
    // keeping the least selection key
    auto eval_chunk = [&](uint32_t tile0, uint32_t h, uint32_t tmask) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * (int)h;
        if (!exact) {
            // fp32 fallback regime: every candidate has S16 ≥ 2^24; any valid domain of the
            // bucket routes the range to fallback_grid through the fit's listing
            const int p = a.tile_pos[tile0 * 32 + row];
            const unsigned long long mask = __ballot(p >= 0 && g == 0);
            if (mask) {
                const int pf = __builtin_amdgcn_readlane(p, __ffsll((long long)mask) - 1);
                bestk = min(bestk, key_miss((uint64_t)kExactLimit, (uint32_t)pf, 0));
            }
            return;
        }
        for (uint32_t tile = tile0; tile < min(tile0 + (uint32_t)kTilesPerStage, a.ntiles); ++tile) {
            if (!((tmask >> (tile - tile0)) & 1u))
                continue;
            // the row's pool position (for the key) and its D4 from the tile-order copy are
            // independent loads; ΣD4² is summed here rather than loaded through the position.
            // (Loading the chunk's four tiles up front saved 1 µs at C2 but took 24 more VGPRs:
            // 4 instead of 6 waves per SIMD cost the C4 quadtree's 65k-range level 21 µs.)
            const int p = a.tile_pos[tile * 32 + row];
            const uint4* dp = reinterpret_cast<const uint4*>(a.tpool + ((size_t)tile * 32 + row) * 32 + g * (PG / 2));
            const uint4 d0 = dp[0], d1 = dp[1];
            const uint32_t dv[PG / 2] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
            uint32_t sd2 = 0, sd1 = 0;
#pragma unroll
            for (int q = 0; q < PG / 2; ++q) {
                sd2 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, dv[q]), __builtin_bit_cast(ushort2_t, dv[q]),
                                             sd2, false);
                sd1 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, dv[q]), __builtin_bit_cast(ushort2_t, kOnes),
                                             sd1, false);
            }
            sd2 = quad_sum(sd2);
            sd1 = quad_sum(sd1);
            const int nsd2 = -(int)sd2; // ΣD4² ≤ 64·1020² < 2^31
            unsigned long long tk = kKeyNone;
            uint32_t tx = 0, ts1 = 0, ts2 = 0;
#pragma unroll
            for (int t = 0; t < T; ++t) {
                uint32_t X = 0;
#pragma unroll
                for (int q = 0; q < PG / 2; ++q) {
                    // pair q of orbit q/2 for transform t (see the lane map above)
                    // t odd: the rotated pairs, rebuilt per transform (a t = 1 copy held across
                    // the loop would take 8 more VGPRs)
                    const int qs = q ^ (t >> 1);
                    const uint32_t dq = (t & 1) ? __builtin_amdgcn_alignbit(dv[qs ^ 1], dv[qs], 16) : dv[qs];
                    X = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, rp[q]), __builtin_bit_cast(ushort2_t, dq),
                                               X, false);
                }
                X = quad_sum(X);
                // S16 = 16Σr² − 8X + ΣD4² ≤ 64·1020² < 2^31: exact in int32
                const int64_t s16 = p >= 0 ? (int64_t)(16 * sr2 - 8 * (int32_t)X - nsd2) : 0;
                const bool ok = p >= 0 && g == 0 && (hit ? (s16 <= a.hitH) : (s16 == target));
                const uint32_t tr = flip ? 4u + ((4u - (uint32_t)t) & 3u) : (uint32_t)t; // the reference's transform
                if constexpr (SORTED) {
                    // lane-local least key; one wave reduction per range at the end
                    const unsigned long long k =
                        ok ? (hit ? key_hit((uint32_t)p, tr) : key_miss((uint64_t)target, (uint32_t)p, TK - 1 - tr))
                           : kKeyNone;
                    if (k < tk) {
                        tk = k;
                        tx = X;
                    }
                } else {
                    const unsigned long long mask = __ballot(ok);
                    if (mask) {
                        const int first = __ffsll((long long)mask) - 1;
                        const int pf = __builtin_amdgcn_readlane(p, first);
                        const unsigned long long k = hit ? key_hit((uint32_t)pf, tr)
                                                         : key_miss((uint64_t)target, (uint32_t)pf, TK - 1 - tr);
                        const uint32_t xf = (uint32_t)__builtin_amdgcn_readlane((int)X, first);
                        const uint32_t s1f = (uint32_t)__builtin_amdgcn_readlane((int)sd1, first);
                        const uint32_t s2f = (uint32_t)__builtin_amdgcn_readlane((int)sd2, first);
                        if (k < tk) {
                            tk = k;
                            tx = xf;
                            ts1 = s1f;
                            ts2 = s2f;
                        }
                    }
                }
            }
            if constexpr (SORTED) {
                ts1 = sd1;
                ts2 = sd2;
            }
            if (tk != kKeyNone) {
                if (tk < bestk) {
                    bestk = tk;
                    bx = tx;
                    bs1 = ts1;
                    bs2 = ts2;
                }
                if constexpr (!SORTED)
                    break;
            }
        }
    };
    if (a.slotbest) {
        // the search merged its splits itself (search_dft, DftArgs::slotbest): the slot's greatest y, the
        // earliest chunk attaining it, its tiles to evaluate and which lane halves attain it — one load, no
        // CSR walk
        if (sb == 0ull)
            return res; // no work item reached the slot: no eligible domain
        vmax = funmap((uint32_t)(sb >> 32));
        if (!(vmax > -1.0e29f))
            return res; // only padding rows: no eligible domain, best_key stays "none"
        set_target();
        const uint32_t tile0 = kSlotBestTileMax - ((uint32_t)sb >> 6), tm = ((uint32_t)sb >> 2) & 0xfu;
        const uint32_t hm = (uint32_t)sb & 3u;
        for (uint32_t h = 0; h < 2; ++h)
            if ((hm >> h) & 1u)
                eval_chunk(tile0, h, tm);
    } else {
        const uint32_t e0 = a.blk_ptr[blk], e1 = a.blk_ptr[blk + 1];
        const uint32_t nent = (e1 - e0) * 2u;
        // the first 64 entries stay in registers for the ballot walk below
        uint2 en0 = make_uint2(0u, 0u);
        for (uint32_t j = lane; j < nent; j += 64) {
            const uint2 v = a.entries[(size_t)a.blk_ent[e0 + j / 2] * 64 + col + 32 * (j & 1)];
            if (j < 64)
                en0 = v;
            vmax = __builtin_fmaxf(vmax, __uint_as_float(v.x));
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            vmax = __builtin_fmaxf(vmax, __uint_as_float(lane_xor(__float_as_uint(vmax), lane, o)));
        vmax = __uint_as_float((uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(vmax))); // wave-uniform
        if (!(vmax > -1.0e29f))
            return res; // only padding rows: no eligible domain, best_key stays "none"
        set_target();
        const uint32_t vbits = __float_as_uint(vmax);
        // only the entries holding the maximum are re-evaluated (usually one): the lanes test 64
        // entries at a time and the wave walks the ballot of matches, so the cost does not grow
        // with the number of domain splits (many splits per block when ranges are sharded)
        for (uint32_t c0 = 0; c0 < nent; c0 += 64) {
            const uint32_t jl = c0 + (uint32_t)lane;
            const uint2 enl = jl >= nent ? make_uint2(0u, 0u)
                              : c0 == 0  ? en0
                                         : a.entries[(size_t)a.blk_ent[e0 + jl / 2] * 64 + col + 32 * (jl & 1)];
            unsigned long long match = __ballot(jl < nent && enl.x == vbits);
            while (match) {
                const int src = __ffsll((long long)match) - 1;
                match &= match - 1;
                const uint32_t j = c0 + (uint32_t)src;
                uint32_t ey = (uint32_t)__builtin_amdgcn_readlane((int)enl.y, src);
                // SORTED entries carry the chunk's tile mask in bits 28..31 (search_dft CHUNKED)
                const uint32_t tmask = SORTED ? (ey >> 28) : 0xfu;
                if constexpr (SORTED)
                    ey &= 0x0fffffffu;
                eval_chunk(ey, j & 1u, tmask);
            }
        }
    }
    const unsigned long long mine = bestk;
    if constexpr (SORTED) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long ok2 = ((unsigned long long)lane_xor((uint32_t)(bestk >> 32), lane, o) << 32) |
                                           lane_xor((uint32_t)bestk, lane, o);
            bestk = ok2 < bestk ? ok2 : bestk;
        }
        // the winner's sums: from the lane that evaluated it (keys are unique per (domain, transform)),
        // broadcast through a ballot
        const unsigned long long own = __ballot(mine == bestk && bestk != kKeyNone);
        if (own) {
            const int src = __ffsll((long long)own) - 1;
            bx = (uint32_t)__builtin_amdgcn_readlane((int)bx, src);
            bs1 = (uint32_t)__builtin_amdgcn_readlane((int)bs1, src);
            bs2 = (uint32_t)__builtin_amdgcn_readlane((int)bs2, src);
        }
    }
    res.bestk = bestk;
    res.bx = bx;
    res.bs1 = bs1;
    res.bs2 = bs2;
    res.sr1 = sr1;
    res.sr2 = (uint32_t)sr2;
    return res;
}

// range r's record from its resolved winner w (every lane holds the same after resolve_dft_eval); rg: the
// range's item, loaded by the caller at the start of the resolve
__device__ inline void resolve_dft_record(const MfmaResolveArgs& a, uint32_t r, const DftResolved& w, int lane,
                                          const frac_grid_item& rg)
{
    if (a.fused_fit) { // the range's record right here: one launch less per run (C2: 5 µs of a 43 µs frame)
        if (lane == 0) {
            a.best_key[r] = w.bestk;
            fit_rstat_range<8>(a.fit, r, w.bestk, make_uint4(w.bx, w.bs1 | (w.sr1 << 16), w.bs2, w.sr2), &rg);
        }
        return;
    }
    if (lane == 0) {
        a.best_key[r] = w.bestk;
        if (a.rstat && w.bestk != kKeyNone)
            a.rstat[r] = make_uint4(w.bx, w.bs1 | (w.sr1 << 16), w.bs2, w.sr2);
    }
}

// the slot's range record: its least key (with T = 8's flipped copy, the lesser of the two) and the
// winner's sums for fit_rstat (every lane holds the same after resolve_dft_eval)
template <bool SORTED>
__device__ inline void resolve_dft_slot(const MfmaResolveArgs& a, uint32_t slot, int lane)
{
    const int ri = a.slot_range[slot];
    if (ri < 0)
        return;
    const frac_grid_item rg = a.fused_fit ? a.fit.ranges[ri] : frac_grid_item{};
    DftResolved w = resolve_dft_eval<SORTED>(a, slot, lane, false);
    if (!SORTED && a.flip_slots) {
        const DftResolved f = resolve_dft_eval<SORTED>(a, slot + a.flip_slots, lane, true);
        if (f.bestk < w.bestk)
            w = f;
    }
    resolve_dft_record(a, (uint32_t)ri, w, lane, rg);
}

// T = 8 with the flipped copies (MfmaResolveArgs::paired): a two-wave workgroup per slot, wave 0
// resolving the slot and wave 1 its flipped copy at the same time (the one-wave form ran the two
// one after the other); wave 0 keeps the lesser key and writes the record
__device__ inline void resolve_dft_pair(const MfmaResolveArgs& a, uint32_t slot, uint32_t wave, int lane)
{
    __shared__ unsigned long long fkey;
    __shared__ uint32_t fsums[5];
    const int ri = a.slot_range[slot]; // the same for both waves: the barrier below is reached by both or neither
    if (ri < 0)
        return;
    const frac_grid_item rg = (a.fused_fit && wave == 0) ? a.fit.ranges[ri] : frac_grid_item{};
    const DftResolved w = resolve_dft_eval<false>(a, slot + wave * a.flip_slots, lane, wave == 1);
    if (wave == 1 && lane == 0) {
        fkey = w.bestk;
        fsums[0] = w.bx;
        fsums[1] = w.bs1;
        fsums[2] = w.bs2;
        fsums[3] = w.sr1;
        fsums[4] = w.sr2;
    }
    __syncthreads();
    if (wave == 0) {
        DftResolved f;
        f.bestk = fkey;
        f.bx = fsums[0];
        f.bs1 = fsums[1];
        f.bs2 = fsums[2];
        f.sr1 = fsums[3];
        f.sr2 = fsums[4];
        resolve_dft_record(a, (uint32_t)ri, f.bestk < w.bestk ? f : w, lane, rg);
    }
}

// One wave per slot, in slot order (the 32 ranges of a block read the same entry lines back to
// back); launched as one- or four-wave workgroups. A grid of fewer, longer-lived waves striding over the slots measured slower (452 vs
// 372 µs at C3 in the SEA tiled form).

template <bool SORTED = false>
__global__ void __launch_bounds__(256, 8) resolve_dft(MfmaResolveArgs a)
{
    apply_plan(a);
    if constexpr (!SORTED) {
        if (a.paired) { // two-wave workgroups: the slot and its flipped copy at once
            const uint32_t slot = blockIdx.x;
            if (slot < a.nslots)
                resolve_dft_pair(a, slot, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), threadIdx.x & 63);
            return;
        }
    }
    // the slot is wave-uniform: readfirstlane lets its loads go through the scalar unit
    const uint32_t slot = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (slot < a.nslots)
        resolve_dft_slot<SORTED>(a, slot, threadIdx.x & 63);
}

} // namespace fracenc
