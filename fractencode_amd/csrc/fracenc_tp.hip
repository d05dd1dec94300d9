// fracenc_tp.hip — the SEA engine's tiled form for n = 8, T = 4 (FRAC_FORM_SEA_MFMA):
// the successive-elimination bound of fracenc_sea.hip applied per tile pair, with the
// exhaustive engine's Fourier MFMA kernel doing the arithmetic.
//
//   * domains of each classifier bucket sorted by ΣD4 into 32-domain tiles (tile_pos), each
//     tile with its [min, max] ΣD4; ranges of each bucket sorted by ΣR into 32-range blocks,
//     groups of 8 blocks per workgroup as in the exhaustive search;
//   * tp_seed: per range the exact least error U_r over the tile nearest its ΣR (any real
//     candidate's error bounds the range's minimum from above);
//   * tp_windows: per group the tiles whose ΣD4 interval meets [min ΣR − D, max ΣR + D],
//     D² = n²·(max(U, H) + 1/2) over the group's ranges: outside it (ΣR − ΣD)²/n² alone
//     exceeds the bound, so no candidate there can win, tie or hit (fracenc_sea.hip);
//   * search_dft<…, CHUNKED> over each group's window, one entry per 4-tile chunk (the tiles
//     are in ΣD4 order, not domain order, so every chunk attaining the maximum is kept and
//     resolve_dft re-derives the least selection key over all of them: ties still go to the
//     earliest domain, then the later transform).
// Records are identical to the exhaustive search's; the cost is data-dependent.
#include "fracenc_common.h"

namespace fracenc {

constexpr int kTpMaxBuckets = 8;

struct TpBuckets {
    uint32_t nb;
    uint32_t tile_first[kTpMaxBuckets], tile_count[kTpMaxBuckets];
    uint32_t dom_begin[kTpMaxBuckets], dom_count[kTpMaxBuckets];   // sorted domain entries
    uint32_t blk_first[kTpMaxBuckets], blk_count[kTpMaxBuckets];
    uint32_t rng_begin[kTpMaxBuckets], rng_count[kTpMaxBuckets];   // sorted ranges
};

// range sort key: (bucket << 17) | ΣR (ΣR = 4Σr ≤ 65280)
__global__ void __launch_bounds__(256) tp_range_keys(const uint8_t* __restrict__ tgt, uint32_t tstride,
                                                     const frac_grid_item* __restrict__ ranges,
                                                     const int32_t* __restrict__ rbucket_idx, uint32_t nr,
                                                     uint32_t* __restrict__ key, uint32_t* __restrict__ idx)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nr)
        return;
    const frac_grid_item rg = ranges[r];
    uint32_t s = 0;
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int x = 0; x < 8; ++x)
            s += tgt[(size_t)(rg.y + y) * tstride + rg.x + x];
    key[r] = ((uint32_t)rbucket_idx[r] << 17) | (4u * s);
    idx[r] = r;
}

// tile rows from the sorted domain order; per tile [min, max] ΣD4 of its valid rows
__global__ void __launch_bounds__(256) tp_build_tiles(TpBuckets bk, const uint32_t* __restrict__ skey,
                                                      const uint32_t* __restrict__ spos, uint32_t ntiles,
                                                      int32_t* __restrict__ tile_pos, uint2* __restrict__ tile_sd)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= ntiles * 32u)
        return;
    const uint32_t tile = gid >> 5, row = gid & 31u;
    uint32_t b = 0;
    while (b + 1 < bk.nb && tile >= bk.tile_first[b] + bk.tile_count[b])
        ++b;
    const uint32_t k = (tile - bk.tile_first[b]) * 32u + row;
    const bool valid = k < bk.dom_count[b];
    tile_pos[gid] = valid ? (int32_t)spos[bk.dom_begin[b] + k] : -1;
    if (row == 0) {
        const uint32_t last = min(k + 31u, bk.dom_count[b] - 1u);
        tile_sd[tile] = valid ? make_uint2(skey[bk.dom_begin[b] + k] & 0x1ffffu,
                                           skey[bk.dom_begin[b] + last] & 0x1ffffu)
                              : make_uint2(0xffffffffu, 0u);
    }
}

// range slots from the sorted range order; per block [min, max] ΣR of its valid slots
__global__ void __launch_bounds__(256) tp_build_slots(TpBuckets bk, const uint32_t* __restrict__ rkey,
                                                      const uint32_t* __restrict__ rord, uint32_t nblocks,
                                                      int32_t* __restrict__ slot_range,
                                                      uint32_t* __restrict__ range_slot, uint2* __restrict__ blk_sr,
                                                      uint32_t* __restrict__ blk_u)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= nblocks * 32u)
        return;
    const uint32_t blk = gid >> 5, col = gid & 31u;
    uint32_t b = 0;
    while (b + 1 < bk.nb && blk >= bk.blk_first[b] + bk.blk_count[b])
        ++b;
    const uint32_t k = (blk - bk.blk_first[b]) * 32u + col;
    const bool valid = k < bk.rng_count[b];
    const uint32_t r = valid ? rord[bk.rng_begin[b] + k] : 0u;
    slot_range[gid] = valid ? (int32_t)r : -1;
    if (valid)
        range_slot[r] = gid;
    if (col == 0) {
        const uint32_t last = min(k + 31u, bk.rng_count[b] - 1u);
        blk_sr[blk] = make_uint2(rkey[bk.rng_begin[b] + k] & 0x1ffffu, rkey[bk.rng_begin[b] + last] & 0x1ffffu);
        blk_u[blk] = 0u;
    }
}

// per range: least exact error over the 32 domains of the tile nearest its ΣR → atomicMax
// into its block's bound (lanes: 16 rows × 4 pixel slices, two rounds, as resolve_dft)
struct TpSeedArgs {
    const uint8_t* tgt;
    uint32_t tstride;
    const frac_grid_item* ranges;
    const uint32_t* range_slot;
    const int32_t* rbucket_idx;
    TpBuckets bk;
    const uint2* tile_sd;
    const int32_t* tile_pos;
    const uint32_t* pool;
    const int32_t* negsd2;
    uint32_t nr;
    uint32_t* blk_u;
};

__global__ void __launch_bounds__(256) tp_seed(TpSeedArgs a)
{
    constexpr int N = 8, NN = 64, PG = 16, T = 4;
    const uint32_t r = blockIdx.x * 4u + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= a.nr)
        return;
    const int b = a.rbucket_idx[r];
    const uint32_t t0 = a.bk.tile_first[b], tn = a.bk.tile_count[b];
    if (tn == 0)
        return; // no domain in the bucket: the search has nothing to bound
    const frac_grid_item rg = a.ranges[r];
    const int rv = (int)a.tgt[(size_t)(rg.y + lane / N) * a.tstride + rg.x + (lane % N)];
    int sr = rv, sr2 = rv * rv;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sr += __shfl_xor(sr, o, 64);
        sr2 += __shfl_xor(sr2, o, 64);
    }
    const uint32_t SR = 4u * (uint32_t)sr;
    // the first tile of the bucket whose max ΣD4 reaches ΣR (else the last)
    uint32_t lo = 0, hi = tn - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        if (a.tile_sd[t0 + mid].y < SR)
            lo = mid + 1;
        else
            hi = mid;
    }
    const uint32_t tile = t0 + lo;
    const int i = lane >> 2, g = lane & 3;
    uint32_t pk[T][PG / 2];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int j = 0; j < PG / 2; ++j) {
            const int k = g * PG + 2 * j;
            const uint32_t l = (uint32_t)__shfl(rv, inv_index<N>(t, k), 64);
            const uint32_t h = (uint32_t)__shfl(rv, inv_index<N>(t, k + 1), 64);
            pk[t][j] = l | (h << 16);
        }
    int64_t best = INT64_MAX;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const int p = a.tile_pos[tile * 32 + 16 * half + i];
        uint32_t dv[PG / 2] = {};
        if (p >= 0) {
            const uint4* dp = reinterpret_cast<const uint4*>(a.pool + (size_t)p * (NN / 2) + g * (PG / 2));
            const uint4 d0 = dp[0], d1 = dp[1];
            dv[0] = d0.x, dv[1] = d0.y, dv[2] = d0.z, dv[3] = d0.w;
            dv[4] = d1.x, dv[5] = d1.y, dv[6] = d1.z, dv[7] = d1.w;
        }
        const int nsd2 = p >= 0 ? a.negsd2[p] : 0;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            uint32_t X = 0;
#pragma unroll
            for (int q = 0; q < PG / 2; ++q)
                X = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, pk[t][q]),
                                           __builtin_bit_cast(ushort2_t, dv[q]), X, false);
            X += (uint32_t)__shfl_xor((int)X, 1, 64);
            X += (uint32_t)__shfl_xor((int)X, 2, 64);
            const int64_t s16 = (int64_t)(16 * sr2 - 8 * (int32_t)X - nsd2);
            if (p >= 0 && s16 < best)
                best = s16;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t ob = __shfl_xor(best, o, 64);
        best = ob < best ? ob : best;
    }
    if (lane == 0) {
        // no valid row cannot happen (the tile holds ≥ 1 domain); S16 < 2^27 fits u32
        const uint32_t u = best == INT64_MAX ? 0xffffffffu : (uint32_t)best;
        atomicMax(&a.blk_u[a.range_slot[r] >> 5], u);
    }
}

// per group of ≤ 8 blocks: the tile window and its chunk count
struct TpWindowArgs {
    const uint4* groups;  // [ngroups] {first block, nblocks, tile_first, tile_count} (static)
    uint32_t ngroups;
    const uint2* blk_sr;
    const uint32_t* blk_u;
    const uint2* tile_sd;
    int64_t hitH;         // −1: no hits
    uint4* work;          // [ngroups] {first block, nblocks, t0, t1}
    uint32_t* nchunks;    // [ngroups]
};

__global__ void __launch_bounds__(256) tp_windows(TpWindowArgs a)
{
    const uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= a.ngroups)
        return;
    const uint4 gr = a.groups[gi];
    uint32_t srlo = 0xffffffffu, srhi = 0, u = 0;
    for (uint32_t k = 0; k < gr.y; ++k) {
        const uint2 s = a.blk_sr[gr.x + k];
        srlo = min(srlo, s.x);
        srhi = max(srhi, s.y);
        u = max(u, a.blk_u[gr.x + k]);
    }
    uint32_t t0 = gr.z, t1 = gr.z + gr.w; // the whole bucket when no bound is known
    if (u != 0xffffffffu && gr.w) {
        const double bound = fmax((double)u, (double)a.hitH) + 0.5;
        // (ΣR − ΣD)² / 64 ≤ bound  ⇔  |ΣR − ΣD| ≤ √(64·bound); +1 keeps the rounding conservative
        const int64_t D = (int64_t)sqrt(64.0 * bound) + 1;
        const int64_t lo = (int64_t)srlo - D, hi = (int64_t)srhi + D;
        uint32_t a0 = 0, a1 = gr.w; // first tile with max ΣD4 ≥ lo
        while (a0 < a1) {
            const uint32_t m = (a0 + a1) / 2;
            if ((int64_t)a.tile_sd[gr.z + m].y < lo)
                a0 = m + 1;
            else
                a1 = m;
        }
        uint32_t b0 = a0, b1 = gr.w; // first tile with min ΣD4 > hi
        while (b0 < b1) {
            const uint32_t m = (b0 + b1) / 2;
            if ((int64_t)a.tile_sd[gr.z + m].x <= hi)
                b0 = m + 1;
            else
                b1 = m;
        }
        t0 = gr.z + a0;
        t1 = gr.z + max(a0, b0);
    }
    a.work[gi] = make_uint4(gr.x, gr.y, t0, t1);
    a.nchunks[gi] = (t1 - t0 + 3) / 4;
}

// per block: entry count = its group's chunk count
__global__ void __launch_bounds__(256) tp_block_counts(const uint2* __restrict__ blk_group,
                                                       const uint32_t* __restrict__ nchunks, uint32_t nblocks,
                                                       uint32_t* __restrict__ cnt)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nblocks)
        cnt[b] = blk_group[b].x == 0xffffffffu ? 0u : nchunks[blk_group[b].x];
}

// CSR block → entry bases ((chunk_offset[group] + c) · 8 + wave) read by resolve_dft
__global__ void __launch_bounds__(256) tp_fill_entries(const uint2* __restrict__ blk_group,
                                                       const uint32_t* __restrict__ choff,
                                                       const uint32_t* __restrict__ blk_ptr, uint32_t nblocks,
                                                       uint32_t* __restrict__ blk_ent)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks)
        return;
    const uint2 gw = blk_group[b];
    if (gw.x == 0xffffffffu)
        return;
    for (uint32_t e = blk_ptr[b], c = 0; e < blk_ptr[b + 1]; ++e, ++c)
        blk_ent[e] = (choff[gw.x] + c) * 8u + gw.y;
}

} // namespace fracenc
