// fracenc_tp.hip — the SEA engine's tiled form for n = 8, T = 4 (FRAC_FORM_SEA_MFMA):
// the successive-elimination bound of fracenc_sea.hip applied per tile pair, with the
// exhaustive engine's Fourier MFMA kernel doing the arithmetic.
//
//   * domains of each classifier bucket sorted by ΣD4 into 32-domain tiles (tile_pos), each
//     tile with its [min, max] ΣD4; ranges of each bucket sorted by ΣR into 32-range blocks,
//     groups of 8 blocks per workgroup as in the exhaustive search;
//   * seed: the Fourier search over one tile per group (the tile nearest its middle block's
//     ΣR), tp_seed_reduce turning each range's maximum into U_r, the least exact error over
//     that tile (any real candidate's error bounds the range's minimum from above);
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

// range sort key: (bucket << 16) | ΣR (ΣR = 4Σr ≤ 65280 < 2^16)
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
    key[r] = ((uint32_t)rbucket_idx[r] << 16) | (4u * s);
    idx[r] = r;
}

// domain sort key (bucket << 16) | ΣD4 straight from the plane — ΣD4 is the domain's pixel sum
// (≤ 256·255 < 2^16) — so the pool is built once, by dft_domain_build, after the sort
__device__ inline uint32_t byte_sum4(uint32_t w)
{
    const uint32_t t = (w & 0x00ff00ffu) + ((w >> 8) & 0x00ff00ffu);
    return (t & 0xffffu) + (t >> 16);
}

__global__ void __launch_bounds__(256) tp_domain_keys(const uint8_t* __restrict__ src, uint32_t sstride,
                                                      const frac_grid_item* __restrict__ doms,
                                                      const uint32_t* __restrict__ porig, uint32_t P,
                                                      const uint32_t* __restrict__ bucket_end, uint32_t nb,
                                                      uint32_t* __restrict__ key, uint32_t* __restrict__ pos)
{
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P)
        return;
    const frac_grid_item d = doms[porig[p]];
    const uint8_t* base = src + (size_t)d.y * sstride + d.x;
    uint32_t sd = 0;
    if ((((uintptr_t)base | sstride) & 7u) == 0) {
#pragma unroll
        for (int y = 0; y < 16; ++y) {
            const uint2* row = reinterpret_cast<const uint2*>(base + (size_t)y * sstride);
            const uint2 a = row[0], b = row[1];
            sd += byte_sum4(a.x) + byte_sum4(a.y) + byte_sum4(b.x) + byte_sum4(b.y);
        }
    } else {
        for (int y = 0; y < 16; ++y)
#pragma unroll
            for (int x = 0; x < 16; ++x)
                sd += base[(size_t)y * sstride + x];
    }
    uint32_t b = 0;
    while (b + 1 < nb && p >= bucket_end[b])
        ++b;
    key[p] = (b << 16) | sd;
    pos[p] = p;
}

// tile rows from the sorted domain order; per tile [min, max] ΣD4 of its valid rows; for
// dft_domain_build<BYPOS>: the tile row of each pool position, the padding rows' fragments
// (b = 0) and epilogue constants, and zeroed tile guards
__global__ void __launch_bounds__(256) tp_build_tiles(TpBuckets bk, const uint32_t* __restrict__ skey,
                                                      const uint32_t* __restrict__ spos, uint32_t ntiles,
                                                      int32_t* __restrict__ tile_pos, uint2* __restrict__ tile_sd,
                                                      uint32_t* __restrict__ row_of, uint4* __restrict__ dtiles,
                                                      uint32_t* __restrict__ dconst, uint2* __restrict__ tguard,
                                                      uint32_t ks)
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
    const uint32_t p = valid ? spos[bk.dom_begin[b] + k] : 0u;
    tile_pos[gid] = valid ? (int32_t)p : -1;
    if (valid) {
        row_of[p] = gid;
    } else {
        for (uint32_t st = 0; st < ks; ++st) // ks fragments per tile (the Fourier form's layout)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                dtiles[((size_t)tile * ks + st) * 64 + row + 32 * h] = make_uint4(0u, 0u, 0u, 0u);
        const uint32_t hh = (row >> 2) & 1u, i = (row & 3u) + 4u * (row >> 3);
        dconst[(size_t)tile * (kDftCS * 4) + hh * 16 + i] = __float_as_uint(kDftPadY);
    }
    if (row == 0)
        tguard[tile] = make_uint2(0u, 0u);
    if (row == 0) {
        const uint32_t last = min(k + 31u, bk.dom_count[b] - 1u);
        tile_sd[tile] = valid ? make_uint2(skey[bk.dom_begin[b] + k] & 0xffffu,
                                           skey[bk.dom_begin[b] + last] & 0xffffu)
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
        blk_sr[blk] = make_uint2(rkey[bk.rng_begin[b] + k] & 0xffffu, rkey[bk.rng_begin[b] + last] & 0xffffu);
        blk_u[blk] = 0u;
    }
}

// seed work: per group the one tile of its bucket nearest the ΣR of its middle block
__global__ void __launch_bounds__(256) tp_seed_work(const uint4* __restrict__ groups, uint32_t ngroups,
                                                    const uint2* __restrict__ blk_sr, const uint2* __restrict__ tile_sd,
                                                    uint4* __restrict__ work)
{
    const uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= ngroups)
        return;
    const uint4 gr = groups[gi];
    const uint2 s = blk_sr[gr.x + gr.y / 2];
    const uint32_t SR = (s.x + s.y) / 2;
    uint32_t lo = 0, hi = gr.w - 1; // first tile whose max ΣD4 reaches SR (else the last)
    while (lo < hi) {
        const uint32_t m = (lo + hi) / 2;
        if (tile_sd[gr.z + m].y < SR)
            lo = m + 1;
        else
            hi = m;
    }
    work[gi] = make_uint4(gr.x, gr.y, gr.z + lo, gr.z + lo + 1);
}

// per block: the seed search's maximum y over the seed tile gives each slot U = 16Σa² − y, the
// least exact error over that tile (exact regime; else no bound); the block's bound is the
// greatest U over its slots (a 32-lane reduction, one writer per block)
__global__ void __launch_bounds__(256) tp_seed_reduce(const uint2* __restrict__ blk_group,
                                                      const uint2* __restrict__ entries,
                                                      const int32_t* __restrict__ slot_range,
                                                      const uint32_t* __restrict__ rconst, uint32_t nblocks,
                                                      uint32_t* __restrict__ blk_u)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= nblocks * 32u) // whole blocks: the 32 lanes of a block leave together
        return;
    const uint32_t b = gid >> 5, col = gid & 31u;
    const uint2 gw = blk_group[b];
    if (gw.x == 0xffffffffu)
        return;
    uint32_t u = 0u;
    if (slot_range[gid] >= 0) {
        const size_t e = ((size_t)gw.x * 8u + gw.y) * 64u + col;
        const float y = fmaxf(__uint_as_float(entries[e].x), __uint_as_float(entries[e + 32].x));
        const int64_t sa16 = (int64_t)rconst[gid];
        // y = 16Σa² − min S16 is exact while min S16 < 2^24 (fracenc_dft.hip)
        u = y > (float)(sa16 - kExactLimit) ? (uint32_t)(sa16 - (int64_t)y) : 0xffffffffu;
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1)
        u = max(u, (uint32_t)__shfl_xor((int)u, o, 64));
    if (col == 0)
        blk_u[b] = u;
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
    uint32_t* pairs;      // [ngroups] block × tile pairs searched (frac_stats)
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
    a.pairs[gi] = gr.y * (t1 - t0);
}

// the totals the host needs in one 16-byte copy: {chunks, block → entry links, Σ pairs (u64)}
__global__ void __launch_bounds__(256) tp_totals(const uint32_t* __restrict__ choff, uint32_t ngroups,
                                                 const uint32_t* __restrict__ blk_ptr, uint32_t nblocks,
                                                 const uint32_t* __restrict__ pairs, uint32_t* __restrict__ tot)
{
    __shared__ unsigned long long part[4];
    unsigned long long s = 0;
    for (uint32_t g = threadIdx.x; g < ngroups; g += blockDim.x)
        s += pairs[g];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63u) == 0)
        part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = part[0] + part[1] + part[2] + part[3];
        tot[0] = choff[ngroups];
        tot[1] = blk_ptr[nblocks];
        tot[2] = (uint32_t)t;
        tot[3] = (uint32_t)(t >> 32);
    }
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
