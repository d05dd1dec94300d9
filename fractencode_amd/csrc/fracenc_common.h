// fracenc_common.h — shared device/host definitions of the MI355X search engine.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fracenc.h"

namespace fracenc {

// Ablation kernels (MFMA-only, VALU-only, no LDS-DMA, no barrier …) produce WRONG results by
// design and exist only to locate time. They are compiled only into a -DFRAC_TUNING build
// (tools/ab_mfma.py); the product library (__graft_entry__.build) holds none of them.
#ifdef FRAC_TUNING
constexpr bool kTuningBuild = true;
#else
constexpr bool kTuningBuild = false;
#endif

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

// Dihedral transforms as the reference's 2×4 affine LUT (image/transform.h:32-41):
//   x' = a0·x + a1·y + a2·(sx−1) + a3·(sy−1),  y' = a4·x + a5·y + a6·(sx−1) + a7·(sy−1)
struct Aff {
    int a0, a1, a2, a3, a4, a5, a6, a7;
};

__host__ __device__ constexpr Aff lut(int t)
{
    switch (t) {
    case 0: return {1, 0, 0, 0, 0, 1, 0, 0};    // Id
    case 1: return {0, 1, 0, 0, -1, 0, 1, 0};   // Rotate_90
    case 2: return {-1, 0, 1, 0, 0, -1, 0, 1};  // Rotate_180
    case 3: return {0, -1, 0, 1, 1, 0, 0, 0};   // Rotate_270
    case 4: return {1, 0, 0, 0, 0, -1, 0, 1};   // Flip
    case 5: return {0, 1, 0, 0, 1, 0, 0, 0};    // Flip_Rotate_90
    case 6: return {-1, 0, 1, 0, 0, 1, 0, 0};   // Flip_Rotate_180
    default: return {0, -1, 0, 1, -1, 0, 1, 0}; // Flip_Rotate_270
    }
}

// Ratio-2 decimate-then-permute (verified there for n = 4, 8, 16):
// SamplerBilinear::sample (image/sampler.h:21-38) of range pixel (x, y) under t reads the
// 2×2 block of the domain whose decimated index is D4[by][bx] with
//   bx = a0·x + a1·y + (a2 + a3)·(n−1),  by = a4·x + a5·y + (a6 + a7)·(n−1).
// fwd(t, pix) = by·n + bx  for pix = y·n + x.
template <int N>
__host__ __device__ constexpr int fwd_index(int t, int pix)
{
    const Aff a = lut(t);
    const int x = pix % N, y = pix / N;
    const int bx = a.a0 * x + a.a1 * y + (a.a2 + a.a3) * (N - 1);
    const int by = a.a4 * x + a.a5 * y + (a.a6 + a.a7) * (N - 1);
    return by * N + bx;
}

// Inverse permutation: the range pixel that meets decimated domain cell q under t.
// The linear part is a signed permutation matrix M, so M^-1 = M^T.
template <int N>
__host__ __device__ constexpr int inv_index(int t, int q)
{
    const Aff a = lut(t);
    const int qx = q % N, qy = q / N;
    const int dx = qx - (a.a2 + a.a3) * (N - 1);
    const int dy = qy - (a.a6 + a.a7) * (N - 1);
    const int px = a.a0 * dx + a.a4 * dy;
    const int py = a.a1 * dx + a.a5 * dy;
    return py * N + px;
}

// Selection key of one candidate, reduced with u64 min (atomicMin or in-thread):
//   hit  (S16 <= H):  (0 << 63) | (pool_position << 3) | t
//   miss:             (1 << 63) | (S16 << 27) | (pool_position << 3) | (T − 1 − t)
// Pool positions preserve the reference's domain order inside a classifier bucket,
// so min(key) = "first hit in (domain, transform) order, else least error with ties
// to the earliest domain and then the later transform"
// (encode/TransformEstimator2.hpp:34-41, encode/transformmatcher.h:55-67).
// Engines that do not track t leave the low 3 bits 0; fit_winner re-derives t.
constexpr unsigned long long kKeyNone = ~0ull;
constexpr unsigned long long kKeyMiss = 1ull << 63;
__host__ __device__ inline uint32_t key_pos(unsigned long long k) { return (uint32_t)((k >> 3) & 0xffffffu); }
__host__ __device__ inline unsigned long long key_miss(uint64_t s16, uint32_t pos, uint32_t tcode)
{
    return kKeyMiss | ((unsigned long long)s16 << 27) | ((unsigned long long)pos << 3) | tcode;
}
__host__ __device__ inline unsigned long long key_hit(uint32_t pos, uint32_t t)
{
    return ((unsigned long long)pos << 3) | t;
}

// Cross-lane exchanges without __shfl_xor's bounds checks (which cost 4 VALU per exchange):
// xor 1 / xor 2 inside quads as DPP quad_perm moves (a VALU operand modifier), larger
// distances as one ds_bpermute on a precomputed byte address. Every lane must be active.
__device__ inline uint32_t quad_xor1(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false); // quad_perm [1,0,3,2]
}
__device__ inline uint32_t quad_xor2(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false); // quad_perm [2,3,0,1]
}
__device__ inline uint32_t quad_sum(uint32_t v)
{
    v += quad_xor1(v);
    return v + quad_xor2(v);
}
__device__ inline uint32_t lane_xor(uint32_t v, int lane, int o)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ o) << 2, (int)v);
}

// S16 = Σ(4r − D4)² is the reference's fp32 error ×16 (image/metrics.h:37-50);
// the fp32 sum is exact iff S16 < 2^24.
constexpr int64_t kExactLimit = 1ll << 24;

enum AuxFlags : uint32_t { kAuxHit = 1u, kAuxFallback = 2u, kAuxEmpty = 4u };

struct RangeAux {
    uint32_t pos;   // winning pool position
    uint32_t flags; // AuxFlags
};

constexpr int kMaxBuckets = 8; // 7 classifier buckets (categories −1..5); 1 without the classifier
// the searches' work lists aim at ≥ this many domain tiles per work item (group of range blocks ×
// domain split): on a small frame the target workgroup count would otherwise cut one 4-tile stage per
// workgroup, every workgroup paying its B-fragment loads and first DMA for one stage (C2: 992
// workgroups of 4 tiles in two rounds), and the resolve scanning one entry per split
constexpr uint32_t kMinTilesPerWork = 8;
// the effective target: at most one work item per kMinTilesPerWork group-tiles
__host__ __device__ inline uint64_t work_target(uint64_t target, uint64_t gtiles)
{
    const uint64_t cap = gtiles / kMinTilesPerWork;
    return cap < 1 ? 1 : (cap < target ? cap : target);
}

// per-bucket layout, passed by value to the fill kernels (or read from a DevPlan)
struct BucketLayout {
    uint32_t nb;
    uint32_t VT;                        // engine pool rows per pool position (T in the sampled form, else 1)
    uint32_t dbeg[kMaxBuckets];         // first pool position of the bucket
    uint32_t dcnt[kMaxBuckets];         // pool positions (domains) in the bucket
    uint32_t rbeg[kMaxBuckets];         // first bucket-sorted range of the bucket
    uint32_t rcnt[kMaxBuckets];         // ranges in the bucket
    uint32_t slot_first[kMaxBuckets];   // first slot of the bucket's ranges (blocks padded to `pad` slots)
    uint32_t tile_first[kMaxBuckets];   // first 32-row tile of the bucket's engine pool rows
};

// A search's layout when the device plans it (the quadtree levels, fracenc_bucket.hip qt_plan):
// the bucket counts never come back to the host, so every count the host would have passed as a
// kernel argument lives here, and the kernels (launched on worst-case grids) read it when their
// args carry a plan pointer.  nr and leaf_base of level k + 1 are written by level k's qt_scatter.
struct DevPlan {
    BucketLayout L;      // the MFMA engine's layout (slot_first = 32 · first block, tile_first)
    uint32_t nr;         // ranges of the level
    uint32_t leaf_base;  // leaves the previous levels emitted
    uint32_t nblocks;    // 32-slot range blocks (without T = 8's flipped copies)
    uint32_t ntiles;     // 32-row domain tiles
    uint32_t nwork;      // search work items (workgroups that do work)
    uint32_t nslots;     // range slots, 32 per block (resolve_dft: without the flipped copies)
    uint32_t flip_slots; // T = 8 Fourier: slot s's flipped copy is s + flip_slots (0: none)
    uint32_t pad_;
};

struct SearchArgs {
    const uint8_t* tgt;
    uint32_t tstride;
    const frac_grid_item* ranges;
    const int32_t* slot_range; // range index per range slot (−1 = padding)
    const uint32_t* pool;      // [P][n²/2] packed u16 pairs of D4
    const int32_t* negsd2;     // [P] −ΣD4²
    const uint4* work;         // per wave: {slot_base, p_begin, p_end, group}
    uint32_t nwork;
    int32_t hitH;              // S16 threshold of a hit (≥ 0), see host compute_hit_limit
    unsigned long long* best_key; // [nr]
};

} // namespace fracenc
