// fracenc_mfma.hip — f16 MFMA search engine (ratio-2 path, n ∈ {2, 4, 8}).
//
// The error of every (range, transform, domain) candidate is an all-pairs dot product
// X = Σ_k copy_t[k]·D4[k], i.e. a GEMM with K = n².  It runs on v_mfma_f32_32x32x16_f16
// with operands chosen so the fp32 accumulator is EXACT and its bit pattern is an
// affine function of the integer result:
//   A (rows, 32 domains per tile)         = D4 − 510            ∈ [−510, 510]   (exact in f16)
//   B (cols, 32 ranges, one transform)    = 128 − copy_t         ∈ [−127, 128]
//   C (init)                              = 1.5·2^23
// Every partial sum lies in [2^23, 2^24) (|Σ| ≤ 64·128·510 < 2^22 for n ≤ 8) where fp32
// has unit spacing, so acc is exact and bits(acc) = 0x4B400000 − Z with
// Z = Σ (r − 128)(D4 − 510).  (Exactness measured on gfx950: tools/ubench.hip.)
// Per candidate the epilogue is ONE v_lshl_add_u32:
//   v = (bits << 3) + e'_d  =  S16 + c_r   (mod 2^32, true value in [0, 2^27))
// with e'_d = ΣD4² − 1024·ΣD4 − 0x58000000 per domain and c_r a per-range constant, so
// the min over domains of v is the min of the reference's error S16 (image/metrics.h).
// Lanes keep per (transform) the running min over domain tiles and the first tile that
// attained it (strict '<' in domain order, encode/TransformEstimator2.hpp:34); hits
// (S16 <= H) collapse to 0.  resolve_mfma then pins the exact domain inside that tile.
#pragma once
#include "fracenc_common.h"
#include "fracenc_kernels.hip" // FitArgs, fit_rstat_range (resolve_dft fuses the fit)

namespace fracenc {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float floatx16_t __attribute__((ext_vector_type(16)));

constexpr uint32_t kMfmaPadConst = 0x70000000u; // e' of padding domains: v ≈ 1.9e9, never wins
constexpr int kTilesPerStage = 4; // domain tiles per LDS stage (double-buffered)
constexpr int kDefaultMfmaVariant = 130; // the minimum over transforms first (128), two v_min3 chains (2)
// n ≤ 4: the row constant as the MFMA's C operand (256, the float-C epilogue below) on top of 130
constexpr int kDefaultMfmaVariant4 = 386;

// VAR bit 256, n ≤ 4 (the float-C epilogue): the B operand is 8·(128 − copy_t) ∈ [−1016, 1024] (exact
// in f16) and the accumulator starts from the domain row's e_d = ΣD4² − 1024·ΣD4 ∈ [−2^22, 0], so
//   acc = e_d − 8Z = S16 − c'_r,   c'_r = 16Σr² − 4080Σr + 8·65280·n² = V0 − rconst   (mfma_range_const)
// exactly: every partial sum is bounded by 2^22 + 8·n²·128·510 ≤ 2^22 + 8.36e6 < 2^24 for n ≤ 4.  The
// epilogue is then the minimum of the accumulators themselves — one v_min3_f32 per two candidates:
// 2 VALU per row at T = 4 instead of 3.5 (T/2 + 1.5, VAR 130) — and the entries hold the float minimum
// as an order-preserving u32 (fmap; 0 stays the hit sentinel, ~0u "no candidate").
__host__ __device__ inline uint32_t fmap(float f)
{
    const uint32_t b = __builtin_bit_cast(uint32_t, f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__host__ __device__ inline float funmap(uint32_t u)
{
    return __builtin_bit_cast(float, (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
constexpr float kFltPadE = 1.0e30f; // e of padding domain rows: never the minimum

template <int N>
struct MfmaGeom {
    static constexpr int NN = N * N;
    static constexpr int KS = (NN + 15) / 16; // K-steps of 16
};

// c_r: v − c_r = S16 for a range with pixel sum Σr and square sum Σr²
// v = V0 − 8Z + ΣD4² − 1024ΣD4  and  −8Z = −8X + 4080Σr + 1024ΣD4 − 8·NN·65280
//   ⇒ v = S16 − 16Σr² + 4080Σr + V0 − 8·NN·65280
// V0 = 2^25 for n ≤ 8 (the offset-binary epilogue); 2^28 for n = 16, where |8Z| < 2^27 and
// ΣD4(D4 − 1024) ≥ −2^26 would take v below zero with 2^25 (search_mfma16)
constexpr int64_t mfma_v0(int NN) { return NN > 64 ? (1ll << 28) : (1ll << 25); }
__host__ __device__ inline uint32_t mfma_range_const(int NN, int64_t sr, int64_t sr2)
{
    return (uint32_t)(int64_t)(-16 * sr2 + 4080 * sr + mfma_v0(NN) - 8ll * NN * 65280);
}

// ---------------------------------------------------------------------------
// mfma_domain_prep: u16 pool → per 32-domain tile the A fragments (lane l holds row
// l&31, k = 16s + 8(l>>5) + j) and the per-lane-half epilogue constants e'.
// One thread per (tile, row).  Rows past a bucket's end are padding.
// ---------------------------------------------------------------------------
struct MfmaDomainPrepArgs {
    const uint32_t* pool;       // [P][NN/2]
    const int32_t* negsd2;      // [P]
    const int32_t* tile_pos;    // [ntiles*32] pool position of each tile row (−1 = padding)
    uint32_t ntiles;
    uint4* dtiles;              // [ntiles][KS][64] 16 B
    uint32_t* dconst;           // [ntiles][2][16]
    const DevPlan* plan = nullptr; // device-planned search: ntiles from the plan (the grid is a bound)
    int fmode = 0;              // the float-C epilogue (VAR 256): dconst = float e_d, padding kFltPadE
    // n = 4 / 16 (mfma_prep): the pool rows and −ΣD4² are built here from the source plane (pool_build's
    // sums per tile row) and written beside the fragments, instead of a pool_build launch before; else read
    const uint8_t* src = nullptr;
    uint32_t sstride = 0;
    const frac_grid_item* doms = nullptr;
    const uint32_t* porig = nullptr;
    uint32_t* pool_out = nullptr;
    int32_t* negsd2_out = nullptr;
};

// D4 row k of pool position p (its domain's plane rows 2k and 2k + 1, 2·n columns) as n/2 words of two u16
// pair sums (pool_build<n>); returns Σ of the row's squares
template <int N>
__device__ inline int build_pool_row(const MfmaDomainPrepArgs& a, const frac_grid_item& d, int k, uint32_t* w)
{
    const uint8_t* r0 = a.src + (size_t)(d.y + 2u * (uint32_t)k) * a.sstride + d.x;
    const uint8_t* r1 = r0 + a.sstride;
    int sq = 0;
    if ((((uintptr_t)r0 | a.sstride) & 3u) == 0) {
#pragma unroll
        for (int q = 0; q < N / 2; ++q) {
            const uint32_t v = pair_sums(reinterpret_cast<const uint32_t*>(r0)[q], reinterpret_cast<const uint32_t*>(r1)[q]);
            const int lo = (int)(v & 0xffffu), hi = (int)(v >> 16);
            sq += lo * lo + hi * hi;
            w[q] = v;
        }
    } else {
#pragma unroll
        for (int q = 0; q < N / 2; ++q) {
            const uint8_t* x = r0 + 4 * q;
            const uint8_t* y = r1 + 4 * q;
            const int lo = (int)x[0] + x[1] + y[0] + y[1], hi = (int)x[2] + x[3] + y[2] + y[3];
            sq += lo * lo + hi * hi;
            w[q] = (uint32_t)lo | ((uint32_t)hi << 16);
        }
    }
    return sq;
}

// n = 16: 16 K-steps per row, one lane each (16-lane groups per tile row): the row's 128 pool words and
// 32 fragment stores split 16 ways (one thread per row was a 128-load chain on 63 workgroups: 39 µs at
// the C4 quadtree's first level); the row sum ΣD4 of the epilogue constant by a 16-lane reduction
__device__ __forceinline__ void mfma_domain_prep16_at(MfmaDomainPrepArgs a, uint32_t gid)
{
    constexpr int N = 16, NN = N * N, KS = MfmaGeom<N>::KS;
    if (a.plan)
        a.ntiles = a.plan->ntiles;
    if (gid >= a.ntiles * 32u * KS) // whole 16-lane row groups leave together
        return;
    const uint32_t rg = gid / KS, s = gid % KS, tile = rg >> 5, row = rg & 31u;
    const int p = a.tile_pos[rg];
    int sumd = 0, sq = 0;
    uint32_t bw[8]; // a.src: this lane's D4 row s, built from the plane (and written to the pool)
    if (a.src && p >= 0) {
        sq = build_pool_row<16>(a, a.doms[a.porig[p]], (int)s, bw);
        uint4* pw = reinterpret_cast<uint4*>(a.pool_out + (size_t)p * (NN / 2) + 8 * s);
        pw[0] = make_uint4(bw[0], bw[1], bw[2], bw[3]);
        pw[1] = make_uint4(bw[4], bw[5], bw[6], bw[7]);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        _Float16 v8[8];
        uint4 w = make_uint4(0x01fe01feu, 0x01fe01feu, 0x01fe01feu, 0x01fe01feu); // padding rows: 510 (0)
        if (p >= 0)
            w = a.src ? make_uint4(bw[4 * h], bw[4 * h + 1], bw[4 * h + 2], bw[4 * h + 3])
                      : *reinterpret_cast<const uint4*>(a.pool + (size_t)p * (NN / 2) + 8 * s + 4 * h);
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int dv = (int)((ww[j >> 1] >> (16 * (j & 1))) & 0xffffu);
            if (p >= 0)
                sumd += dv;
            v8[j] = (_Float16)(dv - 510);
        }
        a.dtiles[((size_t)tile * KS + s) * 64 + row + 32 * h] = __builtin_bit_cast(uint4, v8);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
        sumd += __shfl_xor(sumd, o, 64);
        sq += __shfl_xor(sq, o, 64);
    }
    if (s == 0) {
        if (a.src && p >= 0)
            a.negsd2_out[p] = -sq;
        const int sd2 = p >= 0 ? (a.src ? sq : -a.negsd2[p]) : 0;
        const uint32_t e = p >= 0 ? (uint32_t)(sd2 - 1024 * sumd) + (1u << 28) : kMfmaPadConst;
        const uint32_t hh = (row >> 2) & 1u, i = (row & 3u) + 4u * (row >> 3);
        a.dconst[(size_t)tile * 32 + hh * 16 + i] = e;
    }
}

template <int N>
__device__ __forceinline__ void mfma_domain_prep_at(MfmaDomainPrepArgs a, uint32_t gid)
{
    constexpr int NN = N * N, KS = MfmaGeom<N>::KS;
    if (a.plan)
        a.ntiles = a.plan->ntiles;
    if (gid >= a.ntiles * 32u)
        return;
    const uint32_t tile = gid >> 5, row = gid & 31u;
    const int p = a.tile_pos[gid];
    // the pool row, read whole (16-byte loads where it has a multiple of 4 words) alongside −ΣD4²
    constexpr int K2 = NN / 2, K2R = (K2 + 3) / 4 * 4;
    uint32_t w[K2R];
    int sd2 = 0;
    if (N >= 4 && p >= 0 && a.src) { // the pool row from the plane, written to the pool: N rows of N/2 words
        if constexpr (N >= 4) { // (n = 2 rows are read from pool_build's pool: the host sets src for 4 and 16 only)
            const frac_grid_item d = a.doms[a.porig[p]];
#pragma unroll
            for (int k = 0; k < N; ++k)
                sd2 += build_pool_row<N>(a, d, k, w + k * (N / 2));
            uint32_t* pw = a.pool_out + (size_t)p * K2;
#pragma unroll
            for (int q = 0; q < K2; ++q)
                pw[q] = w[q];
            a.negsd2_out[p] = -sd2;
        }
    } else if (p >= 0) {
        if constexpr (K2 % 4 == 0) {
            const uint4* pr = reinterpret_cast<const uint4*>(a.pool + (size_t)p * K2);
#pragma unroll
            for (int q = 0; q < K2 / 4; ++q) {
                const uint4 v = pr[q];
                w[4 * q] = v.x;
                w[4 * q + 1] = v.y;
                w[4 * q + 2] = v.z;
                w[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < K2; ++q)
                w[q] = a.pool[(size_t)p * K2 + q];
        }
        sd2 = -a.negsd2[p];
    }
    int sumd = 0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            _Float16 v8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 16 * s + 8 * h + j;
                int dv = 510; // padding k (n = 2) and padding rows contribute 0
                if (p >= 0 && k < NN) {
                    dv = (k & 1) ? (int)(w[k >> 1] >> 16) : (int)(w[k >> 1] & 0xffffu);
                    sumd += dv;
                }
                v8[j] = (_Float16)(dv - 510);
            }
            a.dtiles[((size_t)tile * KS + s) * 64 + row + 32 * h] = __builtin_bit_cast(uint4, v8);
        }
    }
    // n ≤ 8: v = (bits(acc) << 3) + e with bits(acc) = 0x4B400000 − Z;  n = 16: v = (int(acc) << 3) + e;
    // the float-C epilogue: e_d itself, the accumulator's start
    uint32_t e = p >= 0 ? (uint32_t)(sd2 - 1024 * sumd) + (N == 16 ? (1u << 28) : (uint32_t)-0x58000000)
                        : kMfmaPadConst;
    if (a.fmode)
        e = __float_as_uint(p >= 0 ? (float)(sd2 - 1024 * sumd) : kFltPadE);
    // row = (i&3) + 8(i>>2) + 4h  ⇔  h = (row>>2)&1, i = (row&3) + 4(row>>3)
    const uint32_t h = (row >> 2) & 1u, i = (row & 3u) + 4u * (row >> 3);
    a.dconst[(size_t)tile * 32 + h * 16 + i] = e;
}

// ---------------------------------------------------------------------------
// mfma_range_prep: B fragments of every range block (32 range slots) and transform:
// lane l holds col l&31 (range slot), k = 16s + 8(l>>5) + j, value 128 − copy_t[k]
// with copy_t[k] = r[inv_t(k)].  One thread per (block, t, s, lane).
// ---------------------------------------------------------------------------
struct MfmaRangePrepArgs {
    const uint8_t* tgt;
    uint32_t tstride;
    const frac_grid_item* ranges;
    const int32_t* slot_range; // [nblocks*32]
    uint32_t nblocks;
    uint32_t T;
    uint4* rfrags;             // [nblocks][T][KS][64]
    uint32_t* rconst;          // [nblocks*32]
    uint32_t* rorb = nullptr;  // dft_range_prep: [nblocks*32][32] pixel pairs in orbit order (resolve_dft)
    uint32_t flip_from = ~0u;  // dft_range_prep: blocks from here on hold their range read through Flip (T = 8)
    const DevPlan* plan = nullptr; // device-planned search: the block count (and flip_from) from the plan
    int fmode = 0;             // mfma_range_prep, the float-C epilogue: B = 8·(128 − copy_t)
    unsigned long long* slotbest = nullptr; // dft_range_prep / mfma_range_prep: [nblocks*32] reset to 0 (the
                                            // searches' merged slot words)
};

// the range-block count of a device-planned search (T = 8 Fourier: the originals and their copies)
__device__ inline void apply_plan(MfmaRangePrepArgs& a, uint32_t copies)
{
    if (!a.plan)
        return;
    a.nblocks = a.plan->nblocks * copies;
    if (a.flip_from != ~0u)
        a.flip_from = a.plan->nblocks;
}

template <int N>
__device__ __forceinline__ void mfma_range_prep_at(MfmaRangePrepArgs a, uint32_t gid)
{
    constexpr int NN = N * N, KS = MfmaGeom<N>::KS;
    apply_plan(a, 1);
    const uint32_t per_block = a.T * KS * 64u;
    if (gid >= a.nblocks * per_block)
        return;
    const uint32_t b = gid / per_block, rem = gid % per_block;
    const uint32_t t = rem / (KS * 64u), s = (rem / 64u) % KS, lane = rem % 64u;
    const uint32_t col = lane & 31u, h = lane >> 5;
    const int ri = a.slot_range[b * 32 + col];
    if (a.slotbest && t == 0 && s == 0 && h == 0)
        a.slotbest[b * 32 + col] = 0ull; // the run's reset of search_mfma's merged slot words
    _Float16 v8[8];
    if (ri >= 0) {
        const frac_grid_item rg = a.ranges[ri];
        int32_t part = 0; // this thread's share of rconst (transform 0 covers every pixel once)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 16 * (int)s + 8 * (int)h + j;
            int rv = 128;
            if (k < NN) {
                const int pix = inv_index<N>((int)t, k);
                rv = a.tgt[(size_t)(rg.y + pix / N) * a.tstride + rg.x + (pix % N)];
                part += 4080 * rv - 16 * rv * rv;
            }
            v8[j] = (_Float16)(a.fmode ? 8 * (128 - rv) : 128 - rv);
        }
        // rconst = −16Σr² + 4080Σr + const (mfma_range_const) mod 2^32: the transform-0 threads add
        // their pixels' terms to the zeroed word, the first of them the constant
        if (t == 0) {
            if (s == 0 && h == 0)
                part += (int32_t)mfma_range_const(NN, 0, 0);
            atomicAdd(&a.rconst[b * 32 + col], (uint32_t)part);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v8[j] = (_Float16)0.0f;
    }
    a.rfrags[((size_t)(b * a.T + t) * KS + s) * 64 + lane] = __builtin_bit_cast(uint4, v8);
}

// mfma_range_prep16: mfma_range_prep at n = 16, one 256-thread workgroup per range block.  The 32
// ranges' pixels are read once into LDS (coalesced byte rows, 8 KiB), each range's constant is a
// wave reduction written directly (no atomics, no zeroed word), and the T·16·64 fragments are
// gathered from LDS and written 16 B per lane.  (The thread-per-fragment form read every pixel T
// times from global memory with byte loads and atomically added 512 partial constants per block.)
// Rows of the LDS image are 260 bytes apart, so the 32 columns of a fragment read hit 32 banks.
constexpr uint32_t kRp16Row = 260;

template <int T>
__device__ __forceinline__ void mfma_range_prep16_at(MfmaRangePrepArgs a, uint32_t b)
{
    constexpr int N = 16, NN = 256, KS = MfmaGeom<16>::KS;
    apply_plan(a, 1);
    if (b >= a.nblocks)
        return;
    __shared__ uint8_t px[32 * kRp16Row];
    __shared__ frac_grid_item slot_rg[32];
    __shared__ int32_t slot_ok[32];
    if (threadIdx.x < 32) {
        const int ri = a.slot_range[b * 32 + threadIdx.x];
        slot_ok[threadIdx.x] = ri >= 0;
        if (ri >= 0)
            slot_rg[threadIdx.x] = a.ranges[ri];
    }
    __syncthreads();
    // 32 ranges × 16 rows: two rows per thread, each 16 bytes (four 4-byte loads when the row is
    // aligned, else byte loads), all independent; an empty slot reads as 128, whose fragment values are 0
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        const uint32_t row = threadIdx.x + 256u * k, col = row >> 4, y = row & 15u;
        uint32_t w[4] = {0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};
        if (slot_ok[col]) {
            const frac_grid_item rg = slot_rg[col];
            const uint8_t* src = a.tgt + (size_t)(rg.y + y) * a.tstride + rg.x;
            if (((uintptr_t)src & 3u) == 0) {
                const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    w[q] = s4[q];
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    w[q] = src[4 * q] | (src[4 * q + 1] << 8) | (src[4 * q + 2] << 16) | ((uint32_t)src[4 * q + 3] << 24);
            }
        }
        uint32_t* dst = reinterpret_cast<uint32_t*>(px + col * kRp16Row + y * N);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            dst[q] = w[q];
    }
    __syncthreads();
    // the range constants: 8 threads per range, 32 pixels each, then a reduction over the 8 lanes
    {
        const uint32_t col = threadIdx.x >> 3, part = threadIdx.x & 7u;
        int32_t s1 = 0, s2 = 0;
#pragma unroll 8
        for (uint32_t q = part * 32; q < part * 32 + 32; ++q) {
            const int32_t v = px[col * kRp16Row + q];
            s1 += v;
            s2 += v * v;
        }
#pragma unroll
        for (int o = 4; o > 0; o >>= 1) {
            s1 += __shfl_xor(s1, o, 64);
            s2 += __shfl_xor(s2, o, 64);
        }
        if (part == 0)
            a.rconst[b * 32 + col] = slot_ok[col] ? mfma_range_const(NN, s1, s2) : 0u;
    }
    // the fragments: output word o = ((t·KS + s)·64 + lane), lane = col + 32h, k = 16s + 8h + j; thread
    // x takes o = x + 256m, so t = m / 4 is a constant of each unrolled step (the permutation affine)
    const uint32_t lane = threadIdx.x & 63u, col = lane & 31u, h = lane >> 5;
#pragma unroll
    for (int m = 0; m < T * KS * 64 / 256; ++m) {
        constexpr int kPerT = KS * 64 / 256; // 4 steps per transform
        const int t = m / kPerT;
        const uint32_t o = threadIdx.x + 256u * (uint32_t)m, s = (o >> 6) % KS;
        _Float16 v8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 16 * (int)s + 8 * (int)h + j;
            const int rv = px[col * kRp16Row + inv_index<N>(t, k)];
            v8[j] = (_Float16)(a.fmode ? 8 * (128 - rv) : 128 - rv);
        }
        a.rfrags[((size_t)b * T * KS) * 64 + o] = __builtin_bit_cast(uint4, v8);
    }
}

// The direct form's preparation in one launch (dft_prep's arrangement): blocks [0, dblocks) build the domain
// tiles (mfma_domain_prep), the rest the range blocks' fragments (mfma_range_prep; n = 16: one block per
// range block), so the two run side by side instead of one after the other.  T: n = 16's transforms (the
// range half's template); the smaller sides read a.T.
template <int N, int T = 0>
__global__ void __launch_bounds__(256) mfma_prep(MfmaDomainPrepArgs d, MfmaRangePrepArgs r, uint32_t dblocks)
{
    if (blockIdx.x < dblocks) {
        if constexpr (N == 16)
            mfma_domain_prep16_at(d, blockIdx.x * blockDim.x + threadIdx.x);
        else
            mfma_domain_prep_at<N>(d, blockIdx.x * blockDim.x + threadIdx.x);
    } else {
        if constexpr (N == 16)
            mfma_range_prep16_at<T>(r, blockIdx.x - dblocks);
        else
            mfma_range_prep_at<N>(r, (blockIdx.x - dblocks) * blockDim.x + threadIdx.x);
    }
}

// ---------------------------------------------------------------------------
// search_mfma<N, T, HITS>: workgroup = 4 waves = 4 range blocks of one bucket; the
// domain tiles [tile_begin, tile_end) of that bucket are staged through LDS and shared.
// ---------------------------------------------------------------------------
struct MfmaSearchArgs {
    const uint4* dtiles;
    const uint4* dconst;   // [ntiles][8] (= [2][16] u32); the Fourier forms pad a tile to kDftCS = 16
    const uint4* rfrags;
    const uint32_t* rconst;
    const uint4* work;     // per WG: {first block, number of blocks (1..4), tile_begin, tile_end}
    uint32_t nwork;
    uint32_t hitH;         // valid when HITS
    uint2* entries;        // [nwork*4][T][64] {min v (0 = hit), tile}
    const DevPlan* plan = nullptr; // device-planned search: workgroups past plan->nwork leave at once
    // search_mfma with entries merged over t (VAR 128 / 256): instead of the entries, per range slot one
    // 64-bit atomicMax per work item, ~v << 32 | (kDirectSlotTileMax − chunk) << 2 | the lane halves of that
    // chunk attaining v — the least v and, among equal v, the earliest chunk (resolve_small reads it)
    unsigned long long* slotbest = nullptr;
};
constexpr uint32_t kDirectSlotTileMax = 0x3fffffffu; // chunk tiles below 2^30

// a workgroup of a device-planned search's worst-case grid with no work item
__device__ inline bool past_plan(const MfmaSearchArgs& a)
{
    return a.plan && blockIdx.x >= a.plan->nwork;
}

// CS: uint4 of epilogue constants per tile (8 = [2][16] u32; the Fourier search pads them to 16, one
// LDS-DMA piece per 4-tile stage, fracenc_dft.hip kDftCS)
template <int KS, uint32_t NTHREADS = 256, uint32_t CS = 8>
__device__ inline void stage_tiles(uint4* dst, const uint4* __restrict__ dtiles, const uint4* __restrict__ dconst,
                                   uint32_t tb, uint32_t nt)
{
    // LDS-DMA (global_load_lds_dwordx4): the LDS image is lane-linear per wave, which is
    // exactly this [A fragments | epilogue constants] stage layout.
    const uint32_t na = nt * KS * 64u, ntot = na + nt * CS;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t i = threadIdx.x; i < ntot; i += NTHREADS) {
        const uint4* src = i < na ? dtiles + (size_t)tb * KS * 64 + i : dconst + (size_t)tb * CS + (i - na);
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(dst + (i - lane)), 16, 0, 0);
    }
}

// The stage hand-off of every LDS-DMA search loop: this wave's own pieces have landed
// (LDS-DMA is counted by vmcnt only), then the workgroup barrier covers the other waves'.
// __syncthreads() alone is not enough: the compiler emits only lgkmcnt(0) before a barrier
// whose preceding DMA it cannot match to a later ds_read (seen at the loop head of
// search_dft: a stage could be read before all of its pieces had landed).
// tests/test_lds_dma.py guards this statically (tools/lds_dma_check.py over the product code
// object); FRAC_TEST_PLAIN_STAGE_BARRIER builds the hazard back in, only for that test's
// negative control (a standalone kernel object, never the product library).
__device__ inline void stage_barrier()
{
#ifndef FRAC_TEST_PLAIN_STAGE_BARRIER
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __syncthreads();
}

template <int N, int T, bool PRIO = false>
__device__ inline floatx16_t mfma_tile(const half8_t (&af)[MfmaGeom<N>::KS], const half8_t (&bt)[MfmaGeom<N>::KS],
                                       const floatx16_t& cinit)
{
    if constexpr (PRIO)
        __builtin_amdgcn_s_setprio(1);
    floatx16_t acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bt[0], cinit, 0, 0, 0);
#pragma unroll
    for (int s = 1; s < MfmaGeom<N>::KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s], bt[s], acc, 0, 0, 0);
    if constexpr (PRIO)
        __builtin_amdgcn_s_setprio(0);
    return acc;
}

// v = (bits << 3) + e' for the 16 rows a lane holds, folded into the running min m
// with two independent v_min3 chains (halves the dependency depth).
template <bool TWO_CHAINS>
__device__ inline uint32_t epilogue_min(const floatx16_t& acc, const uint32_t (&e)[16], uint32_t m)
{
    if constexpr (!TWO_CHAINS) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            m = min(m, (__float_as_uint(acc[i]) << 3) + e[i]);
        return m;
    }
    uint32_t m0 = m, m1 = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
        m0 = min(min(m0, (__float_as_uint(acc[i]) << 3) + e[i]), (__float_as_uint(acc[i + 1]) << 3) + e[i + 1]);
        m1 = min(min(m1, (__float_as_uint(acc[i + 2]) << 3) + e[i + 2]), (__float_as_uint(acc[i + 3]) << 3) + e[i + 3]);
    }
    return min(m0, m1);
}

// Compute the nt tiles of one LDS stage: per tile the A fragments and epilogue constants
// come from LDS; the T transforms are software-pipelined so the MFMAs of transform t+1
// are in flight while the VALU epilogue of transform t runs.
template <int N, int T, int VAR>
__device__ inline void compute_stage(const uint4* __restrict__ la, uint32_t nt, uint32_t lane,
                                     const half8_t (&bf)[T][MfmaGeom<N>::KS], const floatx16_t& cinit,
                                     uint32_t (&cm)[T])
{
    constexpr int KS = MfmaGeom<N>::KS;
    const uint4* lc = la + nt * KS * 64u;
    const uint32_t h = lane >> 5;
    // the float-C epilogue (VAR 256): the stage's running minimum stays a float (one fmap per stage, not per tile)
    float fm = __builtin_inff();
    for (uint32_t q = 0; q < nt; ++q) {
        half8_t af[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s)
            af[s] = __builtin_bit_cast(half8_t, la[(q * KS + s) * 64 + lane]);
        uint32_t e[16];
        auto read_e = [&]() {
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
                const uint4 v = lc[q * 8 + h * 4 + c4];
                e[4 * c4 + 0] = v.x;
                e[4 * c4 + 1] = v.y;
                e[4 * c4 + 2] = v.z;
                e[4 * c4 + 3] = v.w;
            }
        };
        constexpr bool PRIO = (VAR & 32) != 0, LATE_E = (VAR & 64) != 0;
        if constexpr ((VAR & 256) != 0) {
            static_assert(N <= 4, "the float-C epilogue is exact for n <= 4 only");
            read_e();
            floatx16_t c;
#pragma unroll
            for (int i = 0; i < 16; ++i)
                c[i] = __uint_as_float(e[i]);
            floatx16_t acc[T];
#pragma unroll
            for (int t = 0; t < T; ++t)
                acc[t] = mfma_tile<N, T>(af, bf[t], c);
            float m = fm;
            if constexpr (T == 1) {
#pragma unroll
                for (int i = 0; i < 16; i += 2)
                    m = __builtin_fminf(__builtin_fminf(m, acc[0][i]), acc[0][i + 1]);
            } else {
                static_assert(T % 2 == 0 && T >= 4, "T = 4 or 8: three, then pairs, then the last with the running min");
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    float r = __builtin_fminf(__builtin_fminf(acc[0][i], acc[1][i]), acc[2][i]);
#pragma unroll
                    for (int t = 3; t + 1 < T; t += 2)
                        r = __builtin_fminf(__builtin_fminf(r, acc[t][i]), acc[t + 1][i]);
                    m = __builtin_fminf(__builtin_fminf(m, r), acc[T - 1][i]);
                }
            }
            fm = m;
            continue;
        }
        if constexpr (LATE_E) {
            // the first transform's MFMAs wait only for the A fragments; the epilogue
            // constants are read while they run
            const floatx16_t acc0 = mfma_tile<N, T, PRIO>(af, bf[0], cinit);
            __builtin_amdgcn_sched_barrier(0);
            read_e();
            cm[0] = epilogue_min<(VAR & 2) != 0>(acc0, e, cm[0]);
#pragma unroll
            for (int t = 1; t < T; ++t)
                cm[t] = epilogue_min<(VAR & 2) != 0>(mfma_tile<N, T, PRIO>(af, bf[t], cinit), e, cm[t]);
            continue;
        }
        read_e();
        if constexpr ((VAR & 1) != 0) {
            floatx16_t prev = mfma_tile<N, T>(af, bf[0], cinit);
#pragma unroll
            for (int t = 1; t < T; ++t) {
                const floatx16_t cur = mfma_tile<N, T>(af, bf[t], cinit);
                cm[t - 1] = epilogue_min<(VAR & 2) != 0>(prev, e, cm[t - 1]);
                prev = cur;
            }
            cm[T - 1] = epilogue_min<(VAR & 2) != 0>(prev, e, cm[T - 1]);
        } else if constexpr ((VAR & 8) != 0) {
            // ABLATION (tuning only, wrong results): epilogue cut to one value per transform
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const floatx16_t acc = mfma_tile<N, T>(af, bf[t], cinit);
                cm[t] = min(cm[t], (__float_as_uint(acc[0]) << 3) + e[0]);
                asm volatile("" ::"v"(acc));
            }
        } else if constexpr ((VAR & 16) != 0) {
            // ABLATION (tuning only, wrong results): no MFMA, epilogue on operand bits
#pragma unroll
            for (int t = 0; t < T; ++t) {
                floatx16_t acc;
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    acc[i] = __builtin_bit_cast(float, (uint32_t)__builtin_bit_cast(uint4, af[i & (KS - 1)]).x + i + t);
                cm[t] = epilogue_min<false>(acc, e, cm[t]);
            }
        } else if constexpr ((VAR & 128) != 0 && T > 1) {
            // the minimum over the T transforms first, on the accumulator bits (monotone in −Z,
            // one u32 min per candidate: v_min3 over pairs of transforms), then one v_lshl_add per
            // row: T/2 + 1.5 VALU per row instead of 1.5·T.  The lane's entry keeps the merged
            // minimum (slot t = 0) and resolve_mfma evaluates every transform of a matching chunk.
            uint32_t mb[16];
            {
                const floatx16_t a0 = mfma_tile<N, T>(af, bf[0], cinit);
                const floatx16_t a1 = mfma_tile<N, T>(af, bf[1], cinit);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    mb[i] = min(__float_as_uint(a0[i]), __float_as_uint(a1[i]));
            }
#pragma unroll
            for (int t = 2; t < T; t += 2) {
                const floatx16_t x = mfma_tile<N, T>(af, bf[t], cinit);
                const floatx16_t y = mfma_tile<N, T>(af, bf[t + 1], cinit);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    mb[i] = min(min(mb[i], __float_as_uint(x[i])), __float_as_uint(y[i]));
            }
            uint32_t m = cm[0];
#pragma unroll
            for (int i = 0; i < 16; i += 2)
                m = min(min(m, (mb[i] << 3) + e[i]), (mb[i + 1] << 3) + e[i + 1]);
            cm[0] = m;
        } else {
#pragma unroll
            for (int t = 0; t < T; ++t)
                cm[t] = epilogue_min<(VAR & 2) != 0>(mfma_tile<N, T, PRIO>(af, bf[t], cinit), e, cm[t]);
        }
    }
    if constexpr ((VAR & 256) != 0)
        if (nt)
            cm[0] = min(cm[0], fmap(fm));
}

// Schedule variant bits (A/B'd in one process by tools/ab_mfma.py):
//   1: software-pipelined transforms (MFMAs of t+1 in flight during the epilogue of t)
//   2: two independent v_min3 chains in the epilogue
//   4: the two LDS stage buffers are distinct __shared__ objects (the LDS-DMA into one
//      provably does not alias ds_reads of the other, so no vmcnt(0) before each tile)
//   128: the minimum over the transforms on the accumulator bits first (entries merged over
//      t; resolve_mfma with MfmaResolveArgs::merged evaluates every transform of a match)
template <int N, int T, bool HITS, int VAR>
__global__ void __launch_bounds__(256) search_mfma(MfmaSearchArgs a)
{
    static_assert(kTuningBuild || (VAR & (8 | 16)) == 0, "search_mfma ablations exist only in FRAC_TUNING builds");
    if (past_plan(a))
        return;
    constexpr int KS = MfmaGeom<N>::KS;
    constexpr int STAGE = kTilesPerStage * KS * 64 + kTilesPerStage * 8; // uint4 per stage
    // two distinct LDS objects: the stage loop is unrolled by two so the LDS-DMA into
    // one buffer provably does not alias the ds_reads of the other (no vmcnt(0) drain)
    constexpr bool SPLIT = (VAR & 4) != 0;
    __shared__ uint4 lds0[SPLIT ? STAGE : 2 * STAGE];
    __shared__ uint4 lds1[SPLIT ? STAGE : 1];
    uint4* const buf0 = lds0;
    uint4* const buf1 = SPLIT ? lds1 : lds0 + STAGE;
    const uint4 wk = a.work[blockIdx.x];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const bool active = wv < wk.y;
    const uint32_t blk = wk.x + (active ? wv : 0u);

    half8_t bf[T][KS];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            bf[t][s] = __builtin_bit_cast(half8_t, a.rfrags[((size_t)(blk * T + t) * KS + s) * 64 + lane]);
    uint32_t hl = 0;
    if constexpr (HITS) {
        if constexpr ((VAR & 256) != 0) {
            // S16 ≤ H ⟺ acc ≤ H − c'_r = H − V0 + rconst; acc is an integer below 2^24 in magnitude, so
            // the clamped bound is exact in f32
            const int64_t lim = (int64_t)a.hitH - mfma_v0(N * N) + (int64_t)(int32_t)a.rconst[blk * 32 + (lane & 31u)];
            hl = fmap((float)max<int64_t>(-(1ll << 24), min<int64_t>(lim, 1ll << 24)));
        } else {
            hl = a.hitH + a.rconst[blk * 32 + (lane & 31u)];
        }
    }

    floatx16_t cinit;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        cinit[i] = 12582912.0f;
    uint32_t best[T], btile[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        best[t] = 0xffffffffu;
        btile[t] = 0;
    }
    auto finish_stage = [&](const uint32_t (&cm)[T], uint32_t tb) {
#pragma unroll
        for (int t = 0; t < T; ++t) {
            uint32_t m = cm[t];
            if constexpr (HITS)
                m = m <= hl ? 0u : m; // any hit in the chunk: the first-hit chunk wins
            if (m < best[t]) {
                best[t] = m;
                btile[t] = tb;
            }
        }
    };
    const uint32_t nstage = (wk.w - wk.z + kTilesPerStage - 1) / kTilesPerStage;
    auto stage_nt = [&](uint32_t st) { return min((uint32_t)kTilesPerStage, wk.w - (wk.z + st * kTilesPerStage)); };
    if (nstage)
        stage_tiles<KS>(buf0, a.dtiles, a.dconst, wk.z, stage_nt(0));
    for (uint32_t st = 0; st < nstage; st += 2) {
        // even stage: read lds0, prefetch stage st+1 into lds1
        {
            const uint32_t tb = wk.z + st * kTilesPerStage;
            stage_barrier();
            if (st + 1 < nstage)
                stage_tiles<KS>(buf1, a.dtiles, a.dconst, tb + kTilesPerStage, stage_nt(st + 1));
            uint32_t cm[T];
#pragma unroll
            for (int t = 0; t < T; ++t)
                cm[t] = 0xffffffffu;
            compute_stage<N, T, VAR>(buf0, stage_nt(st), lane, bf, cinit, cm);
            finish_stage(cm, tb);
        }
        if (st + 1 < nstage) {
            // odd stage: read lds1, prefetch stage st+2 into lds0
            const uint32_t tb = wk.z + (st + 1) * kTilesPerStage;
            stage_barrier();
            if (st + 2 < nstage)
                stage_tiles<KS>(buf0, a.dtiles, a.dconst, tb + kTilesPerStage, stage_nt(st + 2));
            uint32_t cm[T];
#pragma unroll
            for (int t = 0; t < T; ++t)
                cm[t] = 0xffffffffu;
            compute_stage<N, T, VAR>(buf1, stage_nt(st + 1), lane, bf, cinit, cm);
            finish_stage(cm, tb);
        }
    }
    // merged entries (VAR 128): slot t = 0 only, the one resolve_mfma reads
    constexpr int TW = ((VAR & (128 | 256)) != 0 && T > 1) ? 1 : T;
    if constexpr (TW == 1) {
        if (a.slotbest) {
            // lanes l and l + 32 hold one range slot's two row halves: the lesser v, among equal v the earlier
            // chunk, and which halves attain it there (as search_dft's slot words)
            const uint32_t v0 = best[0], c0 = btile[0];
            const uint32_t v1 = (uint32_t)__shfl_xor((int)v0, 32, 64), c1 = (uint32_t)__shfl_xor((int)c0, 32, 64);
            if (active && lane < 32u) {
                uint32_t tile = c0, hm = 1u;
                if (v1 < v0 || (v1 == v0 && c1 < c0)) {
                    tile = c1;
                    hm = 2u;
                } else if (v1 == v0 && c1 == c0) {
                    hm = 3u;
                }
                const unsigned long long w = ((unsigned long long)~min(v0, v1) << 32) |
                                             ((unsigned long long)(kDirectSlotTileMax - tile) << 2) | hm;
                atomicMax(a.slotbest + (size_t)blk * 32 + lane, w);
            }
            return;
        }
    }
    if (active) {
#pragma unroll
        for (int t = 0; t < TW; ++t)
            a.entries[((size_t)(blockIdx.x * 4u + wv) * T + t) * 64 + lane] = make_uint2(best[t], btile[t]);
    }
}

// ---------------------------------------------------------------------------
// search_mfma16<T, HITS>: the direct form for n = 16 (K = 256: 16 MFMAs per transform and
// tile pair).  |Z| ≤ 256·128·510 < 2^24, so the fp32 accumulation from 0 is exact, but the
// offset-binary epilogue of n ≤ 8 needs |Z| < 2^22: here acc = −Z is converted to an
// integer and v = (int(acc) << 3) + e (e carries V0 = 2^28, mfma_range_const).
//
// A workgroup is 4 waves sharing the LDS stages (2 tiles of 16 KiB + row constants, double
// buffered): Mfma16Shape<T>::BPW range blocks × T / TPW transform groups, each wave holding the B
// fragments of TPW = 2 transforms of its block (128 VGPRs), so every A fragment read from LDS feeds
// two MFMAs.  With one transform per wave (one block × T waves) the LDS read stream matched the
// MFMA stream byte for byte (1 KiB per 32-cycle MFMA per wave, 16 waves per CU: LDS co-bound).
// Entries keep search_mfma's layout, ((work·BPW + block)·T + t)·64 + lane, so resolve_mfma reads
// them unchanged.
// ---------------------------------------------------------------------------
constexpr int kTilesPerStage16 = 2;

template <int T>
struct Mfma16Shape {
    static constexpr int TPW = T >= 2 ? 2 : 1; // transforms per wave
    static constexpr int GPB = T / TPW;        // waves per range block
    static constexpr int BPW = 4 / GPB;        // range blocks per workgroup (4 waves)
    static_assert(GPB * BPW == 4, "4 waves per workgroup");
};
// the host's work lists at n = 16 (build_work / qt_plan): blocks per work item
constexpr uint32_t mfma16_bpw(uint32_t T) { return T >= 8 ? 1u : T >= 2 ? 2u : 4u; }
// target workgroups of an n = 16 search (4 rounds of the 512 resident): a work item's fixed cost —
// 32 KiB of B fragments per wave and the first stage's DMA — stays small beside its tiles
constexpr uint32_t kMfma16TargetWgs = 2048;

template <int T, bool HITS>
__global__ void __launch_bounds__(256, 2) search_mfma16(MfmaSearchArgs a)
{
    using Sh = Mfma16Shape<T>;
    constexpr int KS = MfmaGeom<16>::KS, TPW = Sh::TPW; // 16
    static_assert(mfma16_bpw(T) == (uint32_t)Sh::BPW, "host and kernel agree on the blocks per work item");
    constexpr int STAGE = kTilesPerStage16 * KS * 64 + kTilesPerStage16 * 8;
    if (past_plan(a))
        return;
    __shared__ uint4 lds0[STAGE];
    __shared__ uint4 lds1[STAGE];
    const uint4 wk = a.work[blockIdx.x];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t kb = wv / Sh::GPB, t0 = (wv % Sh::GPB) * TPW;
    const bool active = kb < wk.y; // wave-uniform: a work item with fewer blocks idles its other waves
    const uint32_t blk = wk.x + (active ? kb : 0u);
    half8_t bf[TPW][KS];
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            bf[j][s] = __builtin_bit_cast(half8_t, a.rfrags[((size_t)(blk * T + t0 + j) * KS + s) * 64 + lane]);
    uint32_t hl = 0;
    if constexpr (HITS)
        hl = a.hitH + a.rconst[blk * 32 + (lane & 31u)];
    const floatx16_t zero = {};
    uint32_t best[TPW], btile[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        best[j] = 0xffffffffu;
        btile[j] = 0;
    }
    const uint32_t h = lane >> 5;
    auto compute = [&](const uint4* la, uint32_t nt, uint32_t tb) {
        const uint4* lc = la + nt * KS * 64u;
        for (uint32_t q = 0; q < nt; ++q) {
            floatx16_t acc[TPW];
#pragma unroll
            for (int j = 0; j < TPW; ++j)
                acc[j] = zero;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const half8_t af = __builtin_bit_cast(half8_t, la[(q * KS + s) * 64 + lane]);
#pragma unroll
                for (int j = 0; j < TPW; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf[j][s], acc[j], 0, 0, 0);
            }
            uint32_t e[16];
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
                const uint4 v = lc[q * 8 + h * 4 + c4];
                e[4 * c4 + 0] = v.x;
                e[4 * c4 + 1] = v.y;
                e[4 * c4 + 2] = v.z;
                e[4 * c4 + 3] = v.w;
            }
            // the entry names the tile itself (a chunk of one tile), so resolve_mfma<16> re-reads one tile's
            // rows per match, not a stage's: 3 VALU per tile and transform here against 16 rows of 512 B there
#pragma unroll
            for (int j = 0; j < TPW; ++j) {
                uint32_t cm = 0xffffffffu;
#pragma unroll
                for (int i = 0; i < 16; ++i) // acc: exact integer, |acc| < 2^24
                    cm = min(cm, ((uint32_t)(int32_t)acc[j][i] << 3) + e[i]);
                if constexpr (HITS)
                    cm = cm <= hl ? 0u : cm; // any hit in the tile: the first-hit tile wins
                if (cm < best[j]) {
                    best[j] = cm;
                    btile[j] = tb + q;
                }
            }
        }
    };
    const uint32_t nstage = (wk.w - wk.z + kTilesPerStage16 - 1) / kTilesPerStage16;
    auto stage_nt = [&](uint32_t st) { return min((uint32_t)kTilesPerStage16, wk.w - (wk.z + st * kTilesPerStage16)); };
    // stages of 2 tiles, double buffered; each tile is its own chunk for resolve_mfma
    if (nstage)
        stage_tiles<KS, 256>(lds0, a.dtiles, a.dconst, wk.z, stage_nt(0));
    for (uint32_t st = 0; st < nstage; st += 2) {
        const uint32_t tb = wk.z + st * kTilesPerStage16;
        stage_barrier();
        if (st + 1 < nstage)
            stage_tiles<KS, 256>(lds1, a.dtiles, a.dconst, tb + kTilesPerStage16, stage_nt(st + 1));
        if (active)
            compute(lds0, stage_nt(st), tb);
        if (st + 1 < nstage) {
            stage_barrier();
            if (st + 2 < nstage)
                stage_tiles<KS, 256>(lds0, a.dtiles, a.dconst, tb + 2 * kTilesPerStage16, stage_nt(st + 2));
            if (active)
                compute(lds1, stage_nt(st + 1), tb + kTilesPerStage16);
        }
    }
    if (active)
#pragma unroll
        for (int j = 0; j < TPW; ++j)
            a.entries[(((size_t)blockIdx.x * Sh::BPW + kb) * T + t0 + j) * 64 + lane] = make_uint2(best[j], btile[j]);
}

// ---------------------------------------------------------------------------
// resolve_mfma: one thread per range.  Combines the per-(split, transform, lane-half)
// entries of its block: hits first (the first (domain, transform) in order), else the
// minimum error with ties to the earliest domain and the later transform; the exact
// domain inside a tile is re-derived with integer arithmetic.  Writes the selection
// key consumed by fit_winner.
// ---------------------------------------------------------------------------
struct MfmaResolveArgs {
    const uint8_t* tgt;
    uint32_t tstride;
    const frac_grid_item* ranges;
    const uint32_t* range_slot; // [nr] slot of each range
    const uint32_t* blk_ptr;    // CSR over blocks → entry bases (work*4 + wave)
    const uint32_t* blk_ent;
    const uint2* entries;
    const uint32_t* rconst;     // [nblocks*32]
    const int32_t* tile_pos;    // [ntiles*32]
    uint32_t ntiles;
    const uint32_t* pool;
    const int32_t* negsd2;
    uint32_t nr;
    uint32_t T;
    int64_t hitH;               // −1: no hits
    unsigned long long* best_key;
    // resolve_dft only: waves walk the slots; D4 rows in tile order (dft_domain_build)
    const int32_t* slot_range;  // [nslots] range of each slot, −1 padding
    uint32_t nslots;
    const uint32_t* tpool;      // [ntiles*32][32] D4 pairs in orbit order (dft_domain_build)
    const uint32_t* rorb;       // [nslots][32] range pixel pairs in orbit order (dft_range_prep)
    uint4* rstat = nullptr;     // [nr] the winner's {X_t, ΣD4 | Σr << 16, ΣD4², Σr²} (fit_rstat)
    uint32_t flip_slots = 0;    // T = 8 Fourier: slot s's flipped copy is slot s + flip_slots (0: none)
    int merged = 0;             // resolve_mfma: entries hold the minimum over every transform (search_mfma VAR 128)
    int fmode = 0;              // resolve_mfma: the entries are fmap'd float-C minima (search_mfma VAR 256)
    const DevPlan* plan = nullptr; // device-planned search: nr, ntiles, nslots, flip_slots from the plan
    // resolve_dft: the fit runs in the resolving wave (fit_rstat_range) instead of a fit_rstat launch
    int fused_fit = 0;
    FitArgs fit{};
    // resolve_mfma<16>: the range copies are read back from search_mfma16's B fragments (128 − copy_t,
    // f16) instead of gathered pixel by pixel from the plane
    const uint4* rfrags = nullptr;
    // resolve_dft, T = 8: two-wave workgroups, one slot and its flipped copy each (flip_slots > 0)
    int paired = 0;
    // resolve_dft / resolve_small: per slot the search's own merge of its splits (search_dft with
    // DftArgs::slotbest, search_mfma with MfmaSearchArgs::slotbest), read in place of the entries and their CSR map
    const unsigned long long* slotbest = nullptr;
};

__device__ inline void apply_plan(MfmaResolveArgs& a)
{
    if (!a.plan)
        return;
    a.nr = a.plan->nr;
    a.ntiles = a.plan->ntiles;
    a.nslots = a.plan->nslots;
    a.flip_slots = a.plan->flip_slots;
}

__device__ inline int fwd_rt(const Aff& a, int N, int q)
{
    const int x = q % N, y = q / N;
    return (a.a4 * x + a.a5 * y + (a.a6 + a.a7) * (N - 1)) * N + a.a0 * x + a.a1 * y + (a.a2 + a.a3) * (N - 1);
}

// One wave per range.  Lane l covers tile row i = l>>2 of a candidate entry's lane half
// and slice g = l&3 of the pool row (n²/8 packed u16 pairs), so the 16 rows of a tile are
// evaluated at once with exact integers; a ballot picks the first row (domain order) that
// matches.  Per transform the lane holds its slice of the range's inverse-permuted copy
// (the pixels that meet the slice's domain cells under t, as u16 pairs), so a row is one
// contiguous load of pool words and v_dot2_u32_u16 per word (Σ r·D4 < 2^32 for n ≤ 16).
// Matching entries in a chunk after the tile of the best key so far are skipped: their rows
// are later pool positions of the same bucket, so they can neither win nor tie.
template <int N>
__device__ inline uint32_t range_pix_inv(const uint8_t* __restrict__ tgt, uint32_t tstride, const frac_grid_item& rg,
                                         const Aff& af, int q)
{
    const int qx = q % N, qy = q / N;
    const int dx = qx - (af.a2 + af.a3) * (N - 1), dy = qy - (af.a6 + af.a7) * (N - 1);
    const int px = af.a0 * dx + af.a4 * dy, py = af.a1 * dx + af.a5 * dy;
    return tgt[(size_t)(rg.y + py) * tstride + rg.x + px];
}

template <int N>
__global__ void __launch_bounds__(256) resolve_mfma(MfmaResolveArgs a)
{
    constexpr int NN = N * N, K2 = NN / 2, WPL = K2 >= 4 ? K2 / 4 : 1; // pool words per lane slice
    apply_plan(a);
    const uint32_t r = blockIdx.x * 4u + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= a.nr)
        return;
    const uint32_t slot = a.range_slot[r];
    const uint32_t blk = slot >> 5, col = slot & 31u;
    const uint32_t e0 = a.blk_ptr[blk], e1 = a.blk_ptr[blk + 1];
    // merged entries (search_mfma VAR 128) hold the minimum over every transform in slot t = 0; the
    // other T − 1 slots are never written to with a candidate, so only slot 0 is read (T× fewer loads)
    const uint32_t TE = a.merged ? 1u : a.T;
    const uint32_t nent = (e1 - e0) * TE * 2u;
    // the range, its constant and its transform-0 copy do not depend on the entries: their loads are
    // issued first, so their latency overlaps the entries' (the copy is built below)
    const frac_grid_item rg = a.ranges[r];
    const uint32_t rc = a.rconst[slot];
    const int i = lane >> 2, g = lane & 3;
    constexpr uint32_t kOnes = 0x00010001u;
    // the lane's slice of the copy under transform ct (rebuilt when an entry's t differs)
    uint32_t cp[WPL];
    int ct = -1;
    auto build_copy = [&](int t) {
        if constexpr (N == 16) { // always from the fragments (the host sets rfrags for every n = 16 resolve)
            // words g·WPL … g·WPL + 31 = pixels k = 64g … 64g + 63 of copy_t: fragments s = 4g … 4g + 3,
            // both lane halves h (k = 16s + 8h + j)
#pragma unroll
            for (int sl = 0; sl < 4; ++sl)
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const uint4 f = a.rfrags[((size_t)(blk * a.T + (uint32_t)t) * MfmaGeom<16>::KS + 4 * g + sl) * 64 +
                                             col + 32 * hh];
                    const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const uint32_t lo = (uint32_t)(128 - (int)__builtin_bit_cast(_Float16, (uint16_t)(fw[m] & 0xffffu)));
                        const uint32_t hi = (uint32_t)(128 - (int)__builtin_bit_cast(_Float16, (uint16_t)(fw[m] >> 16)));
                        cp[sl * 8 + hh * 4 + m] = lo | (hi << 16);
                    }
                }
            ct = t;
        } else {
            const Aff af = lut(t);
#pragma unroll
            for (int w = 0; w < WPL; ++w) {
                const int k = g * WPL + w;
                cp[w] = k < K2 ? range_pix_inv<N>(a.tgt, a.tstride, rg, af, 2 * k) |
                                     (range_pix_inv<N>(a.tgt, a.tstride, rg, af, 2 * k + 1) << 16)
                               : 0u;
            }
            ct = t;
        }
    };
    build_copy(0);
    // the entries: the first 128 stay in registers (enr) for the match pass below, which reloads
    // only past them
    uint2 enr0 = make_uint2(0xffffffffu, 0u), enr1 = enr0;
    uint32_t vmin = 0xffffffffu;
    // not unrolled: an unrolled copy kept a dozen iterations' index divisions in flight and set the
    // kernel's register peak (160 VGPRs, 3 waves per SIMD at n = 16); nent is ≤ 128 in the common case
#pragma nounroll
    for (uint32_t j = lane; j < nent; j += 64) {
        const uint32_t e = e0 + j / (2u * TE), t = (j >> 1) % TE, h = j & 1u;
        const uint2 en = a.entries[((size_t)a.blk_ent[e] * a.T + t) * 64 + col + 32 * h];
        if (j < 64)
            enr0 = en;
        else if (j < 128)
            enr1 = en;
        vmin = min(vmin, en.x);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        vmin = min(vmin, (uint32_t)__shfl_xor((int)vmin, o, 64));
    vmin = (uint32_t)__builtin_amdgcn_readfirstlane((int)vmin); // wave-uniform: a scalar register
    if (vmin == 0xffffffffu) { // no eligible domain: best_key stays "none"
        if (a.fused_fit && lane == 0)
            fit_sums_range<N>(a.fit, r, kKeyNone, 0, 0, 0, 0, 0);
        return;
    }
    uint32_t sr2u = 0, sr1u = 0; // Σr², Σr (every pixel meets exactly one domain cell)
#pragma unroll
    for (int w = 0; w < WPL; ++w) {
        sr2u = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cp[w]), __builtin_bit_cast(ushort2_t, cp[w]), sr2u,
                                      false);
        sr1u = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cp[w]), __builtin_bit_cast(ushort2_t, kOnes), sr1u,
                                      false);
    }
    // every quad holds the whole copy: the sums are wave-uniform (scalar registers)
    const int64_t sr2 = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)quad_sum(sr2u));
    const int64_t sr1 = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)quad_sum(sr1u));
    // best S16 (when vmin is not a sentinel): v − c_r, or for the float-C entries acc + c'_r = acc + V0 − c_r
    const int64_t target = a.fmode ? (int64_t)funmap(vmin) + mfma_v0(NN) - (int64_t)(int32_t)rc
                                   : (int64_t)vmin - (int64_t)rc;
    // hits: the sentinel 0 (kernel run with H > 0), or a best error that meets H = 0
    const bool hit = a.hitH >= 0 && (vmin == 0 || target <= a.hitH);
    unsigned long long bestk = kKeyNone;
    uint32_t best_tile = 0xffffffffu;
    int64_t bx = 0, bsd = 0, bsd2 = 0; // the best key's X_t, ΣD4, ΣD4² (the fused fit)
    // only the entries holding the minimum are re-evaluated: the lanes test 64 entries at a
    // time and the wave walks the ballot of matches (the cost does not grow with the splits)
    for (uint32_t c0 = 0; c0 < nent; c0 += 64) {
        const uint32_t jl = c0 + (uint32_t)lane;
        uint2 enl = c0 == 0 ? enr0 : enr1;
        if (c0 >= 128 && jl < nent) {
            const uint32_t e = e0 + jl / (2u * TE), t = (jl >> 1) % TE, h = jl & 1u;
            enl = a.entries[((size_t)a.blk_ent[e] * a.T + t) * 64 + col + 32 * h];
        }
        unsigned long long match = __ballot(jl < nent && enl.x == vmin);
        while (match) {
            const int src = __ffsll((long long)match) - 1;
            match &= match - 1;
            const uint32_t j = c0 + (uint32_t)src;
            const uint32_t t = (j >> 1) % TE, h = j & 1u;
            const uint32_t ctile = (uint32_t)__builtin_amdgcn_readlane((int)enl.y, src);
            if (ctile > best_tile)
                continue;
            const int row = (i & 3) + 8 * (i >> 2) + 4 * (int)h;
            // merged entries: every transform of the chunk; per transform the first matching row in
            // tile order is its least key, and no tile after the best key's can win or tie
            const uint32_t tlo = a.merged ? 0u : t, thi = a.merged ? a.T : t + 1u;
            for (uint32_t tt = tlo; tt < thi; ++tt) {
                if ((int)tt != ct)
                    build_copy((int)tt);
                // the entry names the first tile of the chunk that attained the minimum: scan the
                // chunk's tiles in order; the first matching row is the earliest domain
                constexpr uint32_t CH = N == 16 ? 1u : (uint32_t)kTilesPerStage; // search_mfma16: one-tile chunks
                int pch[CH]; // the chunk's rows' pool positions, loaded together
#pragma unroll
                for (uint32_t q = 0; q < CH; ++q)
                    pch[q] = ctile + q < a.ntiles ? a.tile_pos[(ctile + q) * 32 + row] : -1;
#pragma unroll
                for (uint32_t q = 0; q < CH; ++q) {
                    const uint32_t tile = ctile + q;
                    if (tile >= a.ntiles || tile > best_tile)
                        break;
                    const int p = pch[q];
                    uint32_t d[WPL];
                    if (p >= 0 && g * WPL < K2) {
                        const uint32_t* dp = a.pool + (size_t)p * K2 + g * WPL;
                        if constexpr (WPL % 4 == 0) {
#pragma unroll
                            for (int w = 0; w < WPL; w += 4) {
                                const uint4 v = *reinterpret_cast<const uint4*>(dp + w);
                                d[w] = v.x;
                                d[w + 1] = v.y;
                                d[w + 2] = v.z;
                                d[w + 3] = v.w;
                            }
                        } else {
#pragma unroll
                            for (int w = 0; w < WPL; ++w)
                                d[w] = dp[w];
                        }
                    } else {
#pragma unroll
                        for (int w = 0; w < WPL; ++w)
                            d[w] = 0u;
                    }
                    uint32_t xu = 0;
#pragma unroll
                    for (int w = 0; w < WPL; ++w)
                        xu = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cp[w]),
                                                    __builtin_bit_cast(ushort2_t, d[w]), xu, false);
                    const int64_t X = (int64_t)quad_sum(xu);
                    const int64_t s16 = p >= 0 ? 16 * sr2 - 8 * X - (int64_t)a.negsd2[p] : 0;
                    uint32_t sdu = 0; // ΣD4 of the row (the fused fit)
#pragma unroll
                    for (int w = 0; w < WPL; ++w)
                        sdu = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, d[w]),
                                                     __builtin_bit_cast(ushort2_t, kOnes), sdu, false);
                    const uint32_t sd1 = quad_sum(sdu);
                    const bool ok = p >= 0 && g == 0 && (hit ? (s16 <= a.hitH) : (s16 == target));
                    const unsigned long long mask = __ballot(ok);
                    if (mask) {
                        const int first = __ffsll((long long)mask) - 1; // lowest lane = lowest row of the half
                        const int64_t s16f = __shfl(s16, first, 64);
                        const int pf = __shfl(p, first, 64);
                        const unsigned long long k =
                            hit ? key_hit((uint32_t)pf, tt) : key_miss((uint64_t)s16f, (uint32_t)pf, a.T - 1 - tt);
                        if (k < bestk) {
                            bestk = k;
                            best_tile = tile;
                            bx = (int64_t)(uint32_t)__shfl((int)(uint32_t)X, first, 64);
                            bsd = (int64_t)(uint32_t)__shfl((int)sd1, first, 64);
                            bsd2 = -(int64_t)a.negsd2[pf];
                        }
                        break;
                    }
                }
            }
        }
    }
    if (lane == 0) {
        a.best_key[r] = bestk;
        if (a.fused_fit) // the record right here: no fit_winner launch
            fit_sums_range<N>(a.fit, r, bestk, bx, bsd, sr1, bsd2, sr2);
    }
}

// resolve_small<N> (n ∈ {2, 4}, T ∈ {4, 8}): resolve_mfma restated for rows short enough to sit in one
// lane.  Lane l takes tile row i = l >> 2 of a matching entry's lane half and the transforms t ≡ l (mod 4)
// (t and t + 4 at T = 8), each with the whole pool row (n²/2 ≤ 8 words) against its own copy of the range,
// so a chunk's 4 tiles × 16 rows × T transforms take one pass per tile instead of one per (tile,
// transform); the wave's least selection key picks the first hit in (domain, transform) order, else the
// exact least error with ties to the earliest domain, then the later transform — resolve_mfma's order.
// The first tile holding a match ends the walk (later tiles hold later pool positions).  With
// fused_fit the record is written here (fit_sums_range), from the winning lane's sums.
template <int N>
// 6 waves per SIMD (80 VGPRs, 2 spilled): the kernel is latency-bound, and 4 → 5 → 6 waves took the C4
// quadtree's level 4 from 128 to 110 to 100 µs (tools/gpu_r04_s16.sh)
__global__ void __launch_bounds__(256, 6) resolve_small(MfmaResolveArgs a)
{
    static_assert(N == 2 || N == 4, "one pool row per lane");
    constexpr int NN = N * N, K2 = NN / 2;
    constexpr uint32_t kOnes = 0x00010001u;
    apply_plan(a);
    const uint32_t r = blockIdx.x * 4u + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= a.nr)
        return;
    const uint32_t slot = a.range_slot[r];
    const uint32_t blk = slot >> 5, col = slot & 31u;
    // search_mfma merged the work items per slot itself (MfmaSearchArgs::slotbest): one word, no CSR walk
    const unsigned long long sb = a.slotbest ? a.slotbest[slot] : 0ull;
    uint32_t e0 = 0, nent = 0;
    const uint32_t TE = a.merged ? 1u : a.T;
    uint32_t vmin = 0xffffffffu;
    if (a.slotbest) {
        vmin = sb ? ~(uint32_t)(sb >> 32) : 0xffffffffu;
    } else {
        e0 = a.blk_ptr[blk];
        nent = (a.blk_ptr[blk + 1] - e0) * TE * 2u;
#pragma nounroll
        for (uint32_t j = lane; j < nent; j += 64) { // not unrolled, as in resolve_mfma
            const uint32_t e = e0 + j / (2u * TE), t = (j >> 1) % TE, h = j & 1u;
            vmin = min(vmin, a.entries[((size_t)a.blk_ent[e] * a.T + t) * 64 + col + 32 * h].x);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            vmin = min(vmin, (uint32_t)__shfl_xor((int)vmin, o, 64));
        vmin = (uint32_t)__builtin_amdgcn_readfirstlane((int)vmin); // wave-uniform: a scalar register
    }
    if (vmin == 0xffffffffu) {
        if (a.fused_fit && lane == 0)
            fit_sums_range<N>(a.fit, r, kKeyNone, 0, 0, 0, 0, 0);
        return;
    }
    const frac_grid_item rg = a.ranges[r];
    const int i = lane >> 2, t0 = lane & 3;
    const bool two = a.T == 8;
    // the lane's copies of the range under t0 (and t0 + 4): the pixels meeting pool cells 2k, 2k + 1
    uint32_t cp[2][K2];
    uint32_t sr1u = 0, sr2u = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const Aff af = lut(t0 + 4 * c);
#pragma unroll
        for (int k = 0; k < K2; ++k)
            cp[c][k] = (c == 0 || two) ? range_pix_inv<N>(a.tgt, a.tstride, rg, af, 2 * k) |
                                             (range_pix_inv<N>(a.tgt, a.tstride, rg, af, 2 * k + 1) << 16)
                                       : 0u;
    }
#pragma unroll
    for (int k = 0; k < K2; ++k) {
        sr2u = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cp[0][k]), __builtin_bit_cast(ushort2_t, cp[0][k]),
                                      sr2u, false);
        sr1u = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cp[0][k]), __builtin_bit_cast(ushort2_t, kOnes),
                                      sr1u, false);
    }
    // every lane holds the whole range: the sums are wave-uniform (scalar registers)
    const int64_t sr2 = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)sr2u),
                  sr1 = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)sr1u);
    const int64_t target = a.fmode ? (int64_t)funmap(vmin) + mfma_v0(NN) - (int64_t)(int32_t)a.rconst[slot]
                                   : (int64_t)vmin - (int64_t)a.rconst[slot];
    const bool hit = a.hitH >= 0 && (vmin == 0 || target <= a.hitH);
    unsigned long long bestk = kKeyNone;
    uint32_t best_tile = 0xffffffffu;
    int64_t bx = 0, bsd = 0, bsd2 = 0;
    // the rows of lane half h in chunk `ctile`'s tiles, up to the first holding a match
    auto eval_chunk = [&](uint32_t ctile, uint32_t h) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * (int)h;
        for (uint32_t tile = ctile; tile < min(ctile + (uint32_t)kTilesPerStage, a.ntiles) && tile <= best_tile;
             ++tile) {
            const int p = a.tile_pos[tile * 32 + row];
            uint32_t d[K2];
            if (p >= 0) {
                const uint32_t* dp = a.pool + (size_t)p * K2;
                if constexpr (K2 == 8) {
                    const uint4 v0 = reinterpret_cast<const uint4*>(dp)[0], v1 = reinterpret_cast<const uint4*>(dp)[1];
                    d[0] = v0.x, d[1] = v0.y, d[2] = v0.z, d[3] = v0.w, d[4] = v1.x, d[5] = v1.y, d[6] = v1.z, d[7] = v1.w;
                } else {
#pragma unroll
                    for (int k = 0; k < K2; ++k)
                        d[k] = dp[k];
                }
            } else {
#pragma unroll
                for (int k = 0; k < K2; ++k)
                    d[k] = 0u;
            }
            uint32_t sd1u = 0;
#pragma unroll
            for (int k = 0; k < K2; ++k)
                sd1u = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, d[k]), __builtin_bit_cast(ushort2_t, kOnes),
                                              sd1u, false);
            const int64_t nsd2 = p >= 0 ? (int64_t)a.negsd2[p] : 0;
            unsigned long long mk = kKeyNone; // the lane's least key over its transforms
            int64_t mx = 0;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (c == 1 && !two)
                    break;
                uint32_t xu = 0;
#pragma unroll
                for (int k = 0; k < K2; ++k)
                    xu = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cp[c][k]),
                                                __builtin_bit_cast(ushort2_t, d[k]), xu, false);
                const int64_t s16 = 16 * sr2 - 8 * (int64_t)xu - nsd2;
                const uint32_t tt = (uint32_t)(t0 + 4 * c);
                if (p >= 0 && (hit ? (s16 <= a.hitH) : (s16 == target))) {
                    const unsigned long long k =
                        hit ? key_hit((uint32_t)p, tt) : key_miss((uint64_t)s16, (uint32_t)p, a.T - 1 - tt);
                    if (k < mk) {
                        mk = k;
                        mx = (int64_t)xu;
                    }
                }
            }
            unsigned long long wk = mk; // the wave's least key of the tile
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long ok2 = ((unsigned long long)lane_xor((uint32_t)(wk >> 32), lane, o) << 32) |
                                               lane_xor((uint32_t)wk, lane, o);
                wk = ok2 < wk ? ok2 : wk;
            }
            if (wk != kKeyNone) {
                if (wk < bestk) {
                    const int src2 = __ffsll((long long)__ballot(mk == wk)) - 1;
                    bestk = wk;
                    best_tile = tile;
                    bx = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mx, src2);
                    bsd = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)sd1u, src2);
                    bsd2 = -(int64_t)(int32_t)__builtin_amdgcn_readlane((int)(int32_t)nsd2, src2);
                }
                break; // later tiles of the chunk hold later pool positions
            }
        }
    };
    if (a.slotbest) {
        const uint32_t ctile = kDirectSlotTileMax - ((uint32_t)sb >> 2), hm = (uint32_t)sb & 3u;
        for (uint32_t h = 0; h < 2; ++h)
            if ((hm >> h) & 1u)
                eval_chunk(ctile, h);
    }
    for (uint32_t c0 = 0; c0 < nent; c0 += 64) {
        const uint32_t jl = c0 + (uint32_t)lane;
        uint2 enl = make_uint2(0xffffffffu, 0u);
        if (jl < nent) {
            const uint32_t e = e0 + jl / (2u * TE), t = (jl >> 1) % TE, h = jl & 1u;
            enl = a.entries[((size_t)a.blk_ent[e] * a.T + t) * 64 + col + 32 * h];
        }
        unsigned long long match = __ballot(jl < nent && enl.x == vmin);
        while (match) {
            const int src = __ffsll((long long)match) - 1;
            match &= match - 1;
            const uint32_t j = c0 + (uint32_t)src, h = j & 1u;
            const uint32_t ctile = (uint32_t)__builtin_amdgcn_readlane((int)enl.y, src);
            if (ctile > best_tile)
                continue;
            eval_chunk(ctile, h);
        }
    }
    if (lane == 0) {
        a.best_key[r] = bestk;
        if (a.fused_fit)
            fit_sums_range<N>(a.fit, r, bestk, bx, bsd, sr1, bsd2, sr2);
    }
}

} // namespace fracenc
