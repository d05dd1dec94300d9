// fracenc_bucket.hip — classifier bucketing and the engines' work layout, built on the device.
//
// With BrightnessBlocksClassifier2 a range only meets the domains of its own category
// (Classifier2::compare, encode/Classifier2.cpp:70-81), so the pool is stored bucket-major
// (bucket = category + 1, 0 = category −1) with the domain order kept inside a bucket
// (TransformEstimator2::estimate visits domains in grid order, encode/TransformEstimator2.hpp:31).
// Every per-item step runs here: the bucket key of each domain and range (a stored −1 is
// classified on the item's own plane, as compare() does), a stable radix sort of item indices by
// key (rocPRIM Onesweep: the pool order porig and the bucket-sorted range order), the bucket
// boundaries, and the fills of the per-slot / per-tile / per-range maps the engines read.  The
// host sees only the 2 × 8 bucket counts, from which it derives the small per-bucket layout
// (BucketLayout) and the work lists — no per-item host loop and no per-item transfer.
#include <type_traits>

#include "fracenc_common.h"

namespace fracenc {

constexpr int kMaxBuckets = 8; // 7 classifier buckets (categories −1..5); 1 without the classifier

// per-bucket layout, passed by value to the fill kernels
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

// key = category + 1 of item i; a stored −1 is classified on `plane` (classify_items' arithmetic:
// quadrant sums, u16 for quadrants ≤ 16 wide).  A stored category outside −1..5 raises *err.
// One wave per item (blockDim 256).
__global__ void __launch_bounds__(256) bucket_keys(const frac_grid_item* __restrict__ items, uint32_t n,
                                                   const uint8_t* __restrict__ plane, uint32_t stride,
                                                   uint32_t* __restrict__ key, uint32_t* __restrict__ iota,
                                                   uint32_t* __restrict__ err)
{
    const uint32_t k = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (k >= n)
        return;
    const frac_grid_item it = items[k];
    int cat = it.category;
    if (cat == -1) {
        const uint32_t hw = it.w / 2, hh = it.h / 2;
        uint32_t q[4] = {0u, 0u, 0u, 0u};
        const uint32_t qw = 2 * hw, npx = qw * (2 * hh);
        for (uint32_t p = lane; p < npx; p += 64) {
            const uint32_t px = p % qw, py = p / qw;
            q[(py >= hh ? 2 : 0) + (px >= hw ? 1 : 0)] += plane[(size_t)(it.y + py) * stride + it.x + px];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1)
                q[i] += (uint32_t)__shfl_xor((int)q[i], o, 64);
        if (hw <= 16)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                q[i] &= 0xffffu;
        cat = category4_dev(q[0], q[1], q[2], q[3]);
    }
    if (lane == 0) {
        if (cat < -1 || cat > 5) {
            atomicOr(err, 1u);
            cat = -1;
        }
        key[k] = (uint32_t)(cat + 1);
        iota[k] = k;
    }
}

// The same for items at most 64 rows high: L lanes per item (L = the item height rounded up to
// a power of two), lane j sums the two halves of row j (dword loads and v_dot4 when the row
// and the half width are 4-byte aligned, else bytes), and the group reduces the quadrants.
// 64/L items per wave instead of one.
template <uint32_t L>
__global__ void __launch_bounds__(256) bucket_keys_rows(const frac_grid_item* __restrict__ items, uint32_t n,
                                                        const uint8_t* __restrict__ plane, uint32_t stride,
                                                        uint32_t* __restrict__ key, uint32_t* __restrict__ iota,
                                                        uint32_t* __restrict__ err)
{
    static_assert(L >= 1 && L <= 64 && (L & (L - 1)) == 0, "lanes per item: a power of two up to 64");
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t k = gid / L, j = gid % L;
    frac_grid_item it{0, 0, 0, 0, 0};
    if (k < n)
        it = items[k];
    const uint32_t hw = it.w / 2, hh = it.h / 2;
    uint32_t lo = 0, hi = 0;
    if (k < n && it.category == -1 && j < 2 * hh) {
        const uint8_t* row = plane + (size_t)(it.y + j) * stride + it.x;
        if (((((uintptr_t)row) | hw) & 3u) == 0) {
            for (uint32_t c = 0; c < hw; c += 4) {
                lo = __builtin_amdgcn_udot4(*reinterpret_cast<const uint32_t*>(row + c), 0x01010101u, lo, false);
                hi = __builtin_amdgcn_udot4(*reinterpret_cast<const uint32_t*>(row + hw + c), 0x01010101u, hi, false);
            }
        } else {
            for (uint32_t c = 0; c < hw; ++c) {
                lo += row[c];
                hi += row[hw + c];
            }
        }
    }
    uint32_t q[4] = {j < hh ? lo : 0u, j < hh ? hi : 0u, j < hh ? 0u : lo, j < hh ? 0u : hi};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (uint32_t o = L / 2; o > 0; o >>= 1)
            q[i] += (uint32_t)__shfl_xor((int)q[i], (int)o, 64);
    if (j != 0 || k >= n)
        return;
    int cat = it.category;
    if (cat == -1) {
        if (hw <= 16)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                q[i] &= 0xffffu;
        cat = category4_dev(q[0], q[1], q[2], q[3]);
    }
    if (cat < -1 || cat > 5) {
        atomicOr(err, 1u);
        cat = -1;
    }
    key[k] = (uint32_t)(cat + 1);
    iota[k] = k;
}

// bucket keys of `cnt` items of height h (every item of a grid has the size of the first)
inline void launch_bucket_keys(const frac_grid_item* items, uint32_t cnt, uint32_t h, const uint8_t* plane,
                               uint32_t stride, uint32_t* key, uint32_t* iota, uint32_t* err, hipStream_t s)
{
    auto rows = [&](auto lanes) {
        constexpr uint32_t L = decltype(lanes)::value;
        const uint64_t threads = (uint64_t)cnt * L;
        bucket_keys_rows<L><<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(items, cnt, plane, stride, key, iota, err);
    };
    if (h <= 2)
        rows(std::integral_constant<uint32_t, 2>());
    else if (h <= 4)
        rows(std::integral_constant<uint32_t, 4>());
    else if (h <= 8)
        rows(std::integral_constant<uint32_t, 8>());
    else if (h <= 16)
        rows(std::integral_constant<uint32_t, 16>());
    else if (h <= 32)
        rows(std::integral_constant<uint32_t, 32>());
    else if (h <= 64)
        rows(std::integral_constant<uint32_t, 64>());
    else
        bucket_keys<<<(cnt + 3) / 4, 256, 0, s>>>(items, cnt, plane, stride, key, iota, err);
}

__global__ void __launch_bounds__(256) fill_iota(uint32_t* __restrict__ out, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = i;
}

// first index of each bucket in a sorted key array (lower_bound of b, b = 0..kMaxBuckets): one block
__global__ void __launch_bounds__(64) bucket_bounds(const uint32_t* __restrict__ sorted, uint32_t n,
                                                    uint32_t* __restrict__ first)
{
    const uint32_t b = threadIdx.x;
    if (b > (uint32_t)kMaxBuckets)
        return;
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t m = lo + (hi - lo) / 2;
        if (sorted[m] < b)
            lo = m + 1;
        else
            hi = m;
    }
    first[b] = lo;
}

__device__ inline uint32_t layout_bucket_of_slot(const BucketLayout& L, uint32_t slot)
{
    uint32_t b = 0;
    for (uint32_t k = 1; k < L.nb; ++k)
        b = slot >= L.slot_first[k] ? k : b;
    return b;
}

// range slots (MFMA: 32 per block, VALU: 64 per wave): slot s of bucket b holds the bucket's
// k-th range, k = s − slot_first[b], or −1 (padding); range_slot is the inverse map (may be null)
__global__ void __launch_bounds__(256) fill_range_slots(BucketLayout L, const uint32_t* __restrict__ rord,
                                                        uint32_t nslots, int32_t* __restrict__ slot_range,
                                                        uint32_t* __restrict__ range_slot)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslots)
        return;
    const uint32_t b = layout_bucket_of_slot(L, s);
    const uint32_t k = s - L.slot_first[b];
    int32_t r = -1;
    if (k < L.rcnt[b]) {
        r = (int32_t)rord[L.rbeg[b] + k];
        if (range_slot)
            range_slot[r] = s;
    }
    slot_range[s] = r;
}

// tile rows: row j of bucket b's tiles holds engine pool row VT·dbeg[b] + j, or −1 (padding)
__global__ void __launch_bounds__(256) fill_tile_pos(BucketLayout L, uint32_t nrows, int32_t* __restrict__ tile_pos)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nrows)
        return;
    const uint32_t tile = g >> 5;
    uint32_t b = 0;
    for (uint32_t k = 1; k < L.nb; ++k)
        b = tile >= L.tile_first[k] ? k : b;
    const uint32_t j = g - 32u * L.tile_first[b];
    tile_pos[g] = j < L.VT * L.dcnt[b] ? (int32_t)(L.VT * L.dbeg[b] + j) : -1;
}

// per range: the engine pool rows of its bucket [VT·dbeg, VT·(dbeg + dcnt))
__global__ void __launch_bounds__(256) fill_rbucket(BucketLayout L, const uint32_t* __restrict__ rkey, uint32_t nr,
                                                    uint2* __restrict__ rbucket)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nr)
        return;
    const uint32_t b = rkey[r];
    rbucket[r] = make_uint2(L.VT * L.dbeg[b], L.VT * (L.dbeg[b] + L.dcnt[b]));
}

// ---- quadtree level transitions on the device (frac_encode_quadtree) ----
// A level's record i splits (flag 1) when the level may split and its distance exceeds the
// threshold; the level's leaves are appended, in search order, to the frame's leaf list, and the
// split ranges' four quadrants (top-left, top-right, bottom-left, bottom-right) become the next
// level's ranges in their parents' order.  offs = exclusive scan of the flags.
__global__ void __launch_bounds__(256) qt_flags(const frac_encode_item* __restrict__ out, uint32_t n, int can_split,
                                                double split, uint32_t* __restrict__ flags)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        flags[i] = (can_split && out[i].match.score.distance > split) ? 1u : 0u;
}

// A level's frac_stats counters, added on the device into acc = {rejected, hit, fallback, empty,
// evaluated} (frac_fetch's host loop, restated): an empty range rejects every domain (classifier
// on), a hit rejects the ineligible domains before its own in grid order (porig of its pool
// position minus the eligible ones before it), any other range every domain outside its bucket.
struct QtBuckets {
    uint32_t nb;
    uint32_t beg[kMaxBuckets];
    uint32_t end[kMaxBuckets];
};

__global__ void __launch_bounds__(256) qt_level_stats(const RangeAux* __restrict__ aux,
                                                      const uint32_t* __restrict__ rkey,
                                                      const uint32_t* __restrict__ porig, uint32_t nr, uint64_t nd,
                                                      int classifier, QtBuckets B,
                                                      const unsigned long long* __restrict__ sea_count,
                                                      unsigned long long* __restrict__ acc)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long v[4] = {0ull, 0ull, 0ull, 0ull}; // rejected, hit, fallback, empty
    if (r < nr) {
        const RangeAux ax = aux[r];
        const uint32_t b = classifier ? rkey[r] : 0u;
        if (ax.flags & kAuxEmpty) {
            v[3] = 1;
            v[0] = classifier ? nd : 0ull;
        } else {
            v[2] = (ax.flags & kAuxFallback) ? 1ull : 0ull;
            if (ax.flags & kAuxHit) {
                v[1] = 1;
                if (classifier)
                    v[0] = (unsigned long long)porig[ax.pos] - (ax.pos - B.beg[b]);
            } else if (classifier) {
                v[0] = nd - (B.end[b] - B.beg[b]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            v[i] += (unsigned long long)__shfl_xor((long long)v[i], o, 64);
        if ((threadIdx.x & 63u) == 0 && v[i])
            atomicAdd(&acc[i], v[i]);
    }
    if (sea_count && r == 0)
        atomicAdd(&acc[4], *sea_count);
}

__global__ void __launch_bounds__(256) qt_scatter(const frac_encode_item* __restrict__ out,
                                                  const frac_grid_item* __restrict__ ranges, uint32_t n,
                                                  const uint32_t* __restrict__ flags, const uint32_t* __restrict__ offs,
                                                  frac_encode_item* __restrict__ leaves, uint32_t leaf_base,
                                                  frac_grid_item* __restrict__ next, uint32_t* __restrict__ nsplit)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t o = offs[i];
    if (flags[i]) {
        const frac_grid_item r = ranges[i];
        const uint32_t h = r.w / 2;
        next[4 * o + 0] = frac_grid_item{r.x, r.y, h, h, -1};
        next[4 * o + 1] = frac_grid_item{r.x + h, r.y, h, h, -1};
        next[4 * o + 2] = frac_grid_item{r.x, r.y + h, h, h, -1};
        next[4 * o + 3] = frac_grid_item{r.x + h, r.y + h, h, h, -1};
    } else {
        leaves[leaf_base + (i - o)] = out[i];
    }
    if (i == n - 1)
        *nsplit = o + flags[i];
}

} // namespace fracenc
