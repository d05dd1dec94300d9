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
#include <algorithm>
#include <type_traits>

#include "fracenc_common.h"

namespace fracenc {

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
            if (err)
                atomicOr(err, 1u);
            cat = -1;
        }
        key[k] = (uint32_t)(cat + 1);
        if (iota)
            iota[k] = k;
    }
}

// The same for items at most 64 rows high: L lanes per item (L = the item height rounded up to
// a power of two), lane j sums the two halves of row j (dword loads and v_dot4 when the row
// and the half width are 4-byte aligned, else bytes), and the group reduces the quadrants.
// 64/L items per wave instead of one.
// dn (device-planned quadtree levels): the item count is *dn ≤ n, known only on the device; the
// items [*dn, n) of the worst-case grid get the padding key kPadKey, which sorts after every bucket.
constexpr uint32_t kPadKey = 7; // categories −1..5 are keys 0..6; the 3-bit radix sort keeps 7 last

// one grid's keys (bucket_keys_rows, and either half of bucket_keys_rows2)
struct KeySeg {
    const frac_grid_item* items;
    uint32_t n;
    const uint8_t* plane;
    uint32_t stride;
    uint32_t* key;
    uint32_t* iota;
    uint32_t* err;
    const uint32_t* dn;
};

template <uint32_t L>
__device__ inline void keys_rows_item(const KeySeg& sg, uint32_t gid)
{
    static_assert(L >= 1 && L <= 64 && (L & (L - 1)) == 0, "lanes per item: a power of two up to 64");
    const frac_grid_item* __restrict__ items = sg.items;
    const uint8_t* __restrict__ plane = sg.plane;
    uint32_t* __restrict__ key = sg.key;
    uint32_t* __restrict__ iota = sg.iota;
    uint32_t* __restrict__ err = sg.err;
    const uint32_t n = sg.n, stride = sg.stride;
    const uint32_t* dn = sg.dn;
    const uint32_t k = gid / L, j = gid % L;
    if (dn) {
        const uint32_t nd = min(*dn, n);
        if (k >= nd) {
            if (k < n && j == 0) {
                key[k] = kPadKey;
                if (iota)
                    iota[k] = k;
            }
            return; // whole item groups leave together: the shuffles below see only live lanes
        }
    }
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
        if (err)
            atomicOr(err, 1u);
        cat = -1;
    }
    key[k] = (uint32_t)(cat + 1);
    if (iota)
        iota[k] = k;
}

template <uint32_t L>
__global__ void __launch_bounds__(256) bucket_keys_rows(KeySeg sg)
{
    keys_rows_item<L>(sg, blockIdx.x * blockDim.x + threadIdx.x);
}

// Two grids' keys in one launch (a level's domains, 2n rows high, and its ranges, n rows): blocks
// [0, nb0) take s0 with L0 lanes per item, the rest s1 with L1.  The blocks are whole item groups of
// either grid, so the shuffles stay within one grid.
template <uint32_t L0, uint32_t L1>
__global__ void __launch_bounds__(256) bucket_keys_rows2(KeySeg s0, KeySeg s1, uint32_t nb0)
{
    if (blockIdx.x < nb0)
        keys_rows_item<L0>(s0, blockIdx.x * blockDim.x + threadIdx.x);
    else
        keys_rows_item<L1>(s1, (blockIdx.x - nb0) * blockDim.x + threadIdx.x);
}

// bucket keys of `cnt` items of height h (every item of a grid has the size of the first); dn: the
// device-side count of a worst-case grid of cnt items (items ≤ 64 rows high only)
inline void launch_bucket_keys(const frac_grid_item* items, uint32_t cnt, uint32_t h, const uint8_t* plane,
                               uint32_t stride, uint32_t* key, uint32_t* iota, uint32_t* err, hipStream_t s,
                               const uint32_t* dn = nullptr)
{
    auto rows = [&](auto lanes) {
        constexpr uint32_t L = decltype(lanes)::value;
        const uint64_t threads = (uint64_t)cnt * L;
        bucket_keys_rows<L><<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(
            KeySeg{items, cnt, plane, stride, key, iota, err, dn});
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

// ---- classifier keys from the plane's block sums (round 5) ----
// Classifier2's categories depend on an item's four quadrant sums only (Classifier2.cpp:55-68).  The grids
// the engine classifies on every frame — the C4 run's domains and ranges, the quadtree levels' — are
// q-aligned squares of side 2q, q ∈ {2, 4, 8, 16}, whose quadrants are whole q×q blocks of the plane at
// q-aligned positions.  frame_block_sums sums every such block of a plane once (one thread per 4×4 block,
// 8×8 blocks per wave: 2×2 sums from the bytes, 4×4 from those, 8×8 and 16×16 over lane shuffles), and
// bucket_keys_bs classifies an item with four loads from the pyramid instead of re-reading its 4q² pixels
// (each plane pixel was read 4× by the overlapping stride-q domains).  Items that are not such squares are
// summed from the plane by their own thread.  Sums ≤ 16²·255 < 2^16: u16, exact.
// Rows are padded to an even pitch (4-byte aligned rows).
struct BlockSums {
    uint16_t* s[4] = {nullptr, nullptr, nullptr, nullptr}; // q = 2, 4, 8, 16: [⌊H/q⌋][pitch]
    uint32_t cols[4] = {0, 0, 0, 0};                        // ⌊W/q⌋
    uint32_t rows[4] = {0, 0, 0, 0};                        // ⌊H/q⌋
    uint32_t pitch[4] = {0, 0, 0, 0};                       // cols rounded up to even
};

// the pyramid's layout in one buffer of bs_words(W, H) u16 (+ 2 words of slack)
inline size_t bs_words(uint32_t W, uint32_t H)
{
    size_t n = 2;
    for (uint32_t q = 2; q <= 16; q *= 2)
        n += (size_t)(((W / q) + 1) & ~1u) * (H / q);
    return n;
}
inline BlockSums bs_layout(uint16_t* base, uint32_t W, uint32_t H)
{
    BlockSums b;
    size_t off = 0;
    for (int l = 0; l < 4; ++l) {
        const uint32_t q = 2u << l;
        b.s[l] = base + off;
        b.cols[l] = W / q;
        b.rows[l] = H / q;
        b.pitch[l] = (b.cols[l] + 1) & ~1u;
        off += (size_t)b.pitch[l] * b.rows[l];
    }
    return b;
}

__global__ void __launch_bounds__(256) frame_block_sums(const uint8_t* __restrict__ plane, uint32_t stride, uint32_t W,
                                                        uint32_t H, BlockSums b)
{
    const uint32_t W4c = (W + 3) / 4, H4c = (H + 3) / 4; // 4×4 blocks, the last column / row possibly partial
    const uint32_t nwx = (W4c + 7) / 8;
    const uint32_t wid = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t bx = (wid % nwx) * 8 + (lane & 7u), by = (wid / nwx) * 8 + (lane >> 3);
    if (wid >= nwx * ((H4c + 7) / 8))
        return; // whole waves: the shuffles below see only live lanes
    const uint32_t x0 = 4 * bx, y0 = 4 * by;
    uint32_t r[4] = {0u, 0u, 0u, 0u}; // the block's rows, four pixels each (zero outside the plane)
    if (bx < W4c && by < H4c) {
        const uint8_t* p = plane + (size_t)y0 * stride + x0;
        const bool full = x0 + 4 <= W && y0 + 4 <= H && ((((uintptr_t)p) | stride) & 3u) == 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (full) {
                r[i] = *reinterpret_cast<const uint32_t*>(p + (size_t)i * stride);
            } else if (y0 + i < H) {
                for (uint32_t j = 0; j < 4; ++j)
                    if (x0 + j < W)
                        r[i] |= (uint32_t)p[(size_t)i * stride + j] << (8 * j);
            }
        }
    }
    // q = 2: pixel columns (0, 1) and (2, 3) of row pairs (0, 1) and (2, 3)
    uint32_t s2[4], s4 = 0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t m = j ? 0x01010000u : 0x00000101u;
            s2[2 * i + j] = __builtin_amdgcn_udot4(r[2 * i], m, __builtin_amdgcn_udot4(r[2 * i + 1], m, 0u, false), false);
            s4 += s2[2 * i + j];
        }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t cx = 2 * bx + j, cy = 2 * by + i;
            if (cx < b.cols[0] && cy < b.rows[0])
                b.s[0][(size_t)cy * b.pitch[0] + cx] = (uint16_t)s2[2 * i + j];
        }
    if (bx < b.cols[1] && by < b.rows[1])
        b.s[1][(size_t)by * b.pitch[1] + bx] = (uint16_t)s4;
    // q = 8, 16: sums over 2×2 and 4×4 lanes (lane = 8·(by mod 8) + (bx mod 8))
    uint32_t s8 = s4 + (uint32_t)__shfl_xor((int)s4, 1, 64);
    s8 += (uint32_t)__shfl_xor((int)s8, 8, 64);
    uint32_t s16 = s8 + (uint32_t)__shfl_xor((int)s8, 2, 64);
    s16 += (uint32_t)__shfl_xor((int)s16, 16, 64);
    if ((lane & 9u) == 0 && bx / 2 < b.cols[2] && by / 2 < b.rows[2])
        b.s[2][(size_t)(by / 2) * b.pitch[2] + bx / 2] = (uint16_t)s8;
    if ((lane & 27u) == 0 && bx / 4 < b.cols[3] && by / 4 < b.rows[3])
        b.s[3][(size_t)(by / 4) * b.pitch[3] + bx / 4] = (uint16_t)s16;
}

inline void launch_block_sums(const uint8_t* plane, uint32_t stride, uint32_t W, uint32_t H, uint16_t* out,
                              hipStream_t st)
{
    const uint32_t W4c = (W + 3) / 4, H4c = (H + 3) / 4;
    const uint32_t waves = ((W4c + 7) / 8) * ((H4c + 7) / 8);
    if (waves)
        frame_block_sums<<<(waves + 3) / 4, 256, 0, st>>>(plane, stride, W, H, bs_layout(out, W, H));
}

// the pyramid level a grid of w × h items reads (every item of a grid has one size): q = w / 2 = 2^sh
struct BsLevel {
    const uint16_t* s = nullptr; // nullptr: the grid's items are summed from the plane
    uint32_t pitch = 0, sh = 0;
};
inline BsLevel bs_level(const BlockSums& b, uint32_t w, uint32_t h)
{
    BsLevel v;
    const uint32_t q = w / 2;
    const int l = q == 2 ? 0 : q == 4 ? 1 : q == 8 ? 2 : q == 16 ? 3 : -1;
    if (w == h && l >= 0 && b.s[l]) {
        v.s = b.s[l];
        v.pitch = b.pitch[l];
        v.sh = (uint32_t)l + 1u;
    }
    return v;
}

// one item's key from the grid's pyramid level (or, for an item that is not a q-aligned 2q square of that
// level, from the plane by this thread alone); the padding and error rules of keys_rows_item
__device__ __forceinline__ void keys_bs_item(const KeySeg& sg, const BsLevel& lv, uint32_t k)
{
    if (sg.dn && k >= min(*sg.dn, sg.n)) {
        if (k < sg.n) {
            sg.key[k] = kPadKey;
            if (sg.iota)
                sg.iota[k] = k;
        }
        return;
    }
    if (k >= sg.n)
        return;
    const frac_grid_item it = sg.items[k];
    int cat = it.category;
    if (cat == -1) {
        const uint32_t q = 1u << lv.sh;
        uint32_t qs[4] = {0u, 0u, 0u, 0u};
        if (lv.s && it.w == 2 * q && it.h == 2 * q && ((it.x | it.y) & (q - 1)) == 0) {
            const uint16_t* sp = lv.s + (size_t)(it.y >> lv.sh) * lv.pitch + (it.x >> lv.sh);
            qs[0] = sp[0];
            qs[1] = sp[1];
            qs[2] = sp[lv.pitch];
            qs[3] = sp[lv.pitch + 1];
        } else {
            const uint32_t hw = it.w / 2, hh = it.h / 2;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) { // quadrant by quadrant (constant indices: no private array)
                const uint8_t* p0 = sg.plane + (size_t)(it.y + (qd >> 1) * hh) * sg.stride + it.x + (qd & 1) * hw;
                uint32_t t = 0;
                for (uint32_t py = 0; py < hh; ++py)
                    for (uint32_t px = 0; px < hw; ++px)
                        t += p0[(size_t)py * sg.stride + px];
                qs[qd] = t;
            }
            if (hw <= 16)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    qs[i] &= 0xffffu;
        }
        cat = category4_dev(qs[0], qs[1], qs[2], qs[3]);
    }
    if (cat < -1 || cat > 5) {
        if (sg.err)
            atomicOr(sg.err, 1u);
        cat = -1;
    }
    sg.key[k] = (uint32_t)(cat + 1);
    if (sg.iota)
        sg.iota[k] = k;
}

// both grids' keys from block sums, one thread per item: threads [0, s0.n) take s0, the rest s1
__global__ void __launch_bounds__(256) bucket_keys_bs(KeySeg s0, BsLevel l0, KeySeg s1, BsLevel l1)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < s0.n)
        keys_bs_item(s0, l0, i);
    else
        keys_bs_item(s1, l1, i - s0.n);
}

// d: items dw × dh, r: items rw × rh
inline void launch_bucket_keys_bs(const KeySeg& d, const BlockSums& bd, uint32_t dw, uint32_t dh, const KeySeg& r,
                                  const BlockSums& br, uint32_t rw, uint32_t rh, hipStream_t st)
{
    const uint64_t n = (uint64_t)d.n + r.n;
    if (n)
        bucket_keys_bs<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d, bs_level(bd, dw, dh), r, bs_level(br, rw, rh));
}

// a level's domain keys (items 2h rows high) and range keys (h rows) in one launch when h ∈ {4, 8, 16}
// (the C4 frame and the quadtree's levels), else the two launches of launch_bucket_keys
inline void launch_bucket_keys_pair(const KeySeg& d, uint32_t dh, const KeySeg& r, uint32_t rh, hipStream_t s)
{
    auto pair = [&](auto lanes) {
        constexpr uint32_t L = decltype(lanes)::value; // range rows; the domains take 2L
        const unsigned nb0 = (unsigned)(((uint64_t)d.n * 2 * L + 255) / 256);
        const unsigned nb1 = (unsigned)(((uint64_t)r.n * L + 255) / 256);
        bucket_keys_rows2<2 * L, L><<<nb0 + nb1, 256, 0, s>>>(d, r, nb0);
    };
    if (d.n && r.n && dh == 2 * rh && rh > 2 && rh <= 16 && (rh & (rh - 1)) == 0) {
        if (rh == 4)
            pair(std::integral_constant<uint32_t, 4>());
        else if (rh == 8)
            pair(std::integral_constant<uint32_t, 8>());
        else
            pair(std::integral_constant<uint32_t, 16>());
        return;
    }
    if (d.n)
        launch_bucket_keys(d.items, d.n, dh, d.plane, d.stride, d.key, d.iota, d.err, s, d.dn);
    if (r.n)
        launch_bucket_keys(r.items, r.n, rh, r.plane, r.stride, r.key, r.iota, r.err, s, r.dn);
}

// ---- stable bucket sort of item indices by a 3-bit key (the classifier buckets) ----
// A counting sort in two launches, for at most kMaxBuckets keys: per 1,024-item tile the bucket
// counts (bksort_count), then each tile sums every tile's counts itself — the bucket starts
// (first[b] = the first sorted position of bucket b, first[kMaxBuckets] = the count, what
// bucket_bounds computed from the sorted keys; tile 0 writes them) and its own offset per bucket —
// and scatters its indices in index order (bksort_scatter: wave ballots per key give the rank among
// the earlier lanes).  It replaces rocPRIM's Onesweep for these 7 buckets: no memsets, two launches
// (C4 quadtree: six sorts per frame of ≈33 µs each with Onesweep; round 5 folded the per-bucket scan
// over tiles, bksort_scan, into the scatter up to kBkSelfTiles tiles per sort).  dn (device-planned
// levels): the item count is *dn ≤ n; the grids cover n.
constexpr uint32_t kBkTile = 1024, kBkThreads = 256;

// one sort: keys [n] (or the first *dn of them), per-tile counts scratch, bucket starts, sorted indices
struct BkSeg {
    const uint32_t* keys;
    uint32_t n;
    const uint32_t* dn;
    uint32_t* counts; // [tiles · kMaxBuckets]
    uint32_t* first;  // [kMaxBuckets + 1]
    uint32_t* out;
    uint32_t tiles;   // ⌈n / kBkTile⌉
};

// Two independent sorts per launch (a quadtree level's domains and ranges): blocks [0, s0.tiles) take s0,
// the rest s1 (s1.tiles = 0: one sort).
// (by value, field by field: a reference selected between the two kernel arguments put them in scratch)
__device__ inline BkSeg bk_seg(const BkSeg& s0, const BkSeg& s1, uint32_t& blk)
{
    const bool a = blk < s0.tiles;
    if (!a)
        blk -= s0.tiles;
    BkSeg s;
    s.keys = a ? s0.keys : s1.keys;
    s.n = a ? s0.n : s1.n;
    s.dn = a ? s0.dn : s1.dn;
    s.counts = a ? s0.counts : s1.counts;
    s.first = a ? s0.first : s1.first;
    s.out = a ? s0.out : s1.out;
    s.tiles = a ? s0.tiles : s1.tiles;
    return s;
}

__global__ void __launch_bounds__(kBkThreads) bksort_count(BkSeg s0, BkSeg s1)
{
    __shared__ uint32_t part[kBkThreads / 64][kMaxBuckets];
    uint32_t blk = blockIdx.x;
    const BkSeg s = bk_seg(s0, s1, blk);
    const uint32_t n = s.dn ? min(*s.dn, s.n) : s.n;
    const uint32_t base = blk * kBkTile, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t c[kMaxBuckets] = {};
    for (uint32_t j = 0; j < kBkTile / kBkThreads; ++j) {
        const uint32_t i = base + j * kBkThreads + threadIdx.x;
        const uint32_t k = i < n ? s.keys[i] : (uint32_t)kMaxBuckets;
#pragma unroll
        for (uint32_t b = 0; b < (uint32_t)kMaxBuckets; ++b)
            c[b] += (uint32_t)__builtin_popcountll(__ballot(k == b));
    }
    if (lane == 0)
#pragma unroll
        for (uint32_t b = 0; b < (uint32_t)kMaxBuckets; ++b)
            part[wv][b] = c[b];
    __syncthreads();
    if (threadIdx.x < (uint32_t)kMaxBuckets) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < kBkThreads / 64; ++w)
            t += part[w][threadIdx.x];
        s.counts[blk * kMaxBuckets + threadIdx.x] = t;
    }
}

// one block per sort of kMaxBuckets waves, wave b scanning bucket b: offsets[tile][b] = first[b] + the
// bucket's items in earlier tiles (in place over counts).  Lane l takes a run of ⌈tiles / 64⌉ tiles; the
// lanes' run sums are scanned with shuffles, the buckets' totals meet once in LDS.
__global__ void __launch_bounds__(64 * kMaxBuckets) bksort_scan(BkSeg s0, BkSeg s1)
{
    __shared__ uint32_t tot[kMaxBuckets];
    const BkSeg& s = blockIdx.x == 0 ? s0 : s1;
    const uint32_t ntiles = s.tiles;
    const uint32_t b = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t per = (ntiles + 63) / 64, t0 = min(lane * per, ntiles), t1 = min(t0 + per, ntiles);
    uint32_t run = 0;
    for (uint32_t t = t0; t < t1; ++t)
        run += s.counts[t * kMaxBuckets + b];
    uint32_t inc = run; // inclusive scan over the lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = (uint32_t)__shfl_up((int)inc, o, 64);
        if ((int)lane >= o)
            inc += x;
    }
    if (lane == 63)
        tot[b] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t k = 0; k < b; ++k)
        base += tot[k];
    if (lane == 0) {
        s.first[b] = base;
        if (b == kMaxBuckets - 1)
            s.first[kMaxBuckets] = base + tot[b];
    }
    uint32_t off = base + inc - run;
    for (uint32_t t = t0; t < t1; ++t) {
        const uint32_t c = s.counts[t * kMaxBuckets + b];
        s.counts[t * kMaxBuckets + b] = off;
        off += c;
    }
}

// SELF: the tile sums every tile's counts itself (above); else bksort_scan turned them into offsets.  The
// sums read every tile's counts in every tile — quadratic in the tiles, so only for sorts of at most
// kBkSelfTiles tiles
constexpr uint32_t kBkSelfTiles = 512;
template <bool SELF>
__global__ void __launch_bounds__(kBkThreads) bksort_scatter(BkSeg s0, BkSeg s1)
{
    __shared__ uint32_t wcnt[kBkThreads / 64][kMaxBuckets];
    __shared__ uint32_t run[kMaxBuckets];
    __shared__ uint32_t sums[kBkThreads / 64][2 * kMaxBuckets];
    uint32_t blk = blockIdx.x;
    const BkSeg s = bk_seg(s0, s1, blk);
    const uint32_t n = s.dn ? min(*s.dn, s.n) : s.n;
    const uint32_t base = blk * kBkTile, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    if constexpr (!SELF) {
        if (threadIdx.x < (uint32_t)kMaxBuckets)
            run[threadIdx.x] = s.counts[blk * kMaxBuckets + threadIdx.x];
    } else {
        // every tile's counts: per bucket the total and the part in the tiles before this one
        uint32_t tot[kMaxBuckets] = {}, bef[kMaxBuckets] = {};
        for (uint32_t t = threadIdx.x; t < s.tiles; t += kBkThreads)
#pragma unroll
            for (uint32_t b = 0; b < (uint32_t)kMaxBuckets; ++b) {
                const uint32_t c = s.counts[t * kMaxBuckets + b];
                tot[b] += c;
                bef[b] += t < blk ? c : 0u;
            }
#pragma unroll
        for (uint32_t b = 0; b < (uint32_t)kMaxBuckets; ++b)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                tot[b] += (uint32_t)__shfl_xor((int)tot[b], o, 64);
                bef[b] += (uint32_t)__shfl_xor((int)bef[b], o, 64);
            }
        if (lane == 0)
#pragma unroll
            for (uint32_t b = 0; b < (uint32_t)kMaxBuckets; ++b) {
                sums[wv][b] = tot[b];
                sums[wv][kMaxBuckets + b] = bef[b];
            }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t start = 0;
            for (uint32_t b = 0; b < (uint32_t)kMaxBuckets; ++b) {
                uint32_t tb = 0, bb = 0;
                for (uint32_t w = 0; w < kBkThreads / 64; ++w) {
                    tb += sums[w][b];
                    bb += sums[w][kMaxBuckets + b];
                }
                if (blk == 0)
                    s.first[b] = start;
                run[b] = start + bb;
                start += tb;
            }
            if (blk == 0)
                s.first[kMaxBuckets] = start;
        }
        __syncthreads();
    }
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (uint32_t j = 0; j < kBkTile / kBkThreads; ++j) {
        const uint32_t i = base + j * kBkThreads + threadIdx.x;
        const uint32_t k = i < n ? s.keys[i] : (uint32_t)kMaxBuckets;
        uint32_t mine = 0; // the rank among this wave's earlier lanes of the same key
#pragma unroll
        for (uint32_t b = 0; b < (uint32_t)kMaxBuckets; ++b) {
            const unsigned long long m = __ballot(k == b);
            if (k == b)
                mine = (uint32_t)__builtin_popcountll(m & below);
            if (lane == 0)
                wcnt[wv][b] = (uint32_t)__builtin_popcountll(m);
        }
        __syncthreads();
        if (k < (uint32_t)kMaxBuckets) {
            uint32_t pos = run[k] + mine;
            for (uint32_t w = 0; w < wv; ++w)
                pos += wcnt[w][k];
            s.out[pos] = i;
        }
        __syncthreads();
        if (threadIdx.x < (uint32_t)kMaxBuckets)
            for (uint32_t w = 0; w < kBkThreads / 64; ++w)
                run[threadIdx.x] += wcnt[w][threadIdx.x];
        __syncthreads();
    }
}

inline BkSeg bk_seg_of(const uint32_t* keys, uint32_t n, const uint32_t* dn, uint32_t* counts, uint32_t* first,
                       uint32_t* out)
{
    return BkSeg{keys, n, dn, counts, first, out, std::max<uint32_t>((n + kBkTile - 1) / kBkTile, 1u)};
}

// the launches for one or two sorts (s1.tiles = 0: one): two, or three above kBkSelfTiles tiles per sort
inline void launch_bucket_sorts(const BkSeg& s0, const BkSeg& s1, hipStream_t st)
{
    const uint32_t nt = s0.tiles + s1.tiles;
    bksort_count<<<nt, kBkThreads, 0, st>>>(s0, s1);
    if (s0.tiles <= kBkSelfTiles && s1.tiles <= kBkSelfTiles) {
        bksort_scatter<true><<<nt, kBkThreads, 0, st>>>(s0, s1);
    } else {
        bksort_scan<<<s1.tiles ? 2 : 1, 64 * kMaxBuckets, 0, st>>>(s0, s1);
        bksort_scatter<false><<<nt, kBkThreads, 0, st>>>(s0, s1);
    }
}

inline void launch_bucket_sort(const uint32_t* keys, uint32_t n, const uint32_t* dn, uint32_t* counts, uint32_t* first,
                               uint32_t* out, hipStream_t s)
{
    BkSeg none{};
    launch_bucket_sorts(bk_seg_of(keys, n, dn, counts, first, out), none, s);
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
// plan (device-planned levels): the level's range count is plan->nr ≤ n, the grid and the scan
// cover the worst case n, and the items past plan->nr get flag 0.
__global__ void __launch_bounds__(256) qt_flags(const frac_encode_item* __restrict__ out, uint32_t n, int can_split,
                                                double split, uint32_t* __restrict__ flags,
                                                const DevPlan* __restrict__ plan = nullptr)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nl = plan ? min(plan->nr, n) : n;
    if (i < n)
        flags[i] = (i < nl && can_split && out[i].match.score.distance > split) ? 1u : 0u;
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
                                                      unsigned long long* __restrict__ acc,
                                                      const DevPlan* __restrict__ plan = nullptr, uint32_t shards = 1,
                                                      uint32_t stride = 5)
{
    // the block's sums, then one atomic per counter per block into shard blockIdx % shards (stride words
    // apart): a few hundred blocks adding into one word serialise there (24 µs per C4 level); the host
    // sums the shards
    __shared__ unsigned long long part[4][4];
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (plan)
        nr = plan->nr;
    // a bucket's pool positions: from the plan's layout (global memory, indexed by the range's bucket:
    // a per-thread copy of the table would be indexed dynamically, i.e. live in scratch), else from B
    auto dbeg = [&](uint32_t b) { return plan ? plan->L.dbeg[b] : B.beg[b]; };
    auto dcnt = [&](uint32_t b) { return plan ? plan->L.dcnt[b] : B.end[b] - B.beg[b]; };
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
                    v[0] = (unsigned long long)porig[ax.pos] - (ax.pos - dbeg(b));
            } else if (classifier) {
                v[0] = nd - dcnt(b);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            v[i] += (unsigned long long)__shfl_xor((long long)v[i], o, 64);
        if ((threadIdx.x & 63u) == 0)
            part[threadIdx.x >> 6][i] = v[i];
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const unsigned long long t = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] +
                                     part[3][threadIdx.x];
        if (t)
            atomicAdd(&acc[(blockIdx.x % shards) * stride + threadIdx.x], t);
    }
    if (sea_count && r == 0)
        atomicAdd(&acc[4], *sea_count);
}

// plan / next (device-planned levels): the level's count and leaf base come from plan, and the
// next level's (4·nsplit ranges, leaves so far) go to next — the host never reads them per level.
__global__ void __launch_bounds__(256) qt_scatter(const frac_encode_item* __restrict__ out,
                                                  const frac_grid_item* __restrict__ ranges, uint32_t n,
                                                  const uint32_t* __restrict__ flags, const uint32_t* __restrict__ offs,
                                                  frac_encode_item* __restrict__ leaves, uint32_t leaf_base,
                                                  frac_grid_item* __restrict__ next, uint32_t* __restrict__ nsplit,
                                                  const DevPlan* __restrict__ plan = nullptr,
                                                  DevPlan* __restrict__ next_plan = nullptr)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (plan) {
        n = min(plan->nr, n);
        leaf_base = plan->leaf_base;
        if (n == 0 && i == 0) { // an empty level: nothing splits, nothing is emitted
            next_plan->nr = 0;
            next_plan->leaf_base = leaf_base;
        }
    }
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
    if (i == n - 1) {
        const uint32_t ns = o + flags[i];
        if (nsplit)
            *nsplit = ns;
        if (next_plan) {
            next_plan->nr = 4 * ns;
            next_plan->leaf_base = leaf_base + n - ns;
        }
    }
}

// ---- the level transition of a device-planned quadtree level in two launches ----
// (qt_level_stats + qt_flags + a scan + qt_scatter restated): per 1,024-range tile the split count and
// the level's counters (qt_split_count), then per tile its prefix over the earlier tiles' counts (the
// first tile also writes the next level's count and leaf base) and the tile's leaves and quadrants in
// index order (qt_split_emit, the ranks from wave ballots as in bksort_scatter; a separate one-wave scan
// launch cost 4.9 µs per level).  A range splits when the level may split and its distance
// exceeds the threshold; leaves keep the search order, quadrants their parents' order.
struct QtSplitArgs {
    const frac_encode_item* out;  // the level's records
    const frac_grid_item* ranges; // the level's ranges
    const DevPlan* plan;          // nr, leaf_base of this level; layout (stats)
    DevPlan* next;                // receives the next level's nr and leaf_base
    uint32_t nmax;                // the grid's bound
    int can_split;
    double split;
    uint32_t* tcount;             // [tiles] splits per tile (qt_split_emit sums the earlier ones)
    frac_encode_item* leaves;     // device memory, or the caller's pinned host buffer (written over PCIe)
    frac_qt_leaf* leaves32 = nullptr; // instead of `leaves`: the 32-byte leaves (frac_encode_quadtree_leaves)
    uint32_t dcols = 0;           // leaves32: columns of the level's domain grid createUniformGrid(W, H, 2n, n)
    uint32_t leaf_cap;            // leaves past it are not written (the caller's capacity)
    frac_grid_item* next_ranges;
    // the level's frac_stats counters (qt_level_stats), when acc is not null
    const RangeAux* aux;
    const uint32_t* rkey;
    const uint32_t* porig;
    uint64_t nd;
    int classifier;
    unsigned long long* acc;
    uint32_t shards, stride;
};

// a leaf record in 32 bytes (frac_qt_leaf): the winner's domain as its index in the level's domain grid
__host__ __device__ inline frac_qt_leaf qt_leaf_of(const frac_encode_item& r, uint32_t dcols)
{
    const uint32_t n = r.w, lg = n ? 31u - (uint32_t)__builtin_clz(n) : 0u;
    const uint32_t d = r.match.sw ? (r.match.y / n) * dcols + r.match.x / n : FRAC_QT_NO_DOMAIN;
    frac_qt_leaf l;
    l.x = (uint16_t)r.x;
    l.y = (uint16_t)r.y;
    l.code = (d & 0xffffffu) | (((uint32_t)r.match.score.transform & 15u) << 24) | (lg << 28);
    l.contrast = r.match.score.contrast;
    l.brightness = r.match.score.brightness;
    l.distance = r.match.score.distance;
    return l;
}

__device__ inline bool qt_splits(const QtSplitArgs& a, uint32_t i, uint32_t n)
{
    return i < n && a.can_split && a.out[i].match.score.distance > a.split;
}

__global__ void __launch_bounds__(kBkThreads) qt_split_count(QtSplitArgs a)
{
    __shared__ uint32_t wc[kBkThreads / 64];
    __shared__ unsigned long long part[kBkThreads / 64][4];
    const uint32_t n = min(a.plan->nr, a.nmax);
    const uint32_t base = blockIdx.x * kBkTile, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t c = 0;
    unsigned long long v[4] = {0ull, 0ull, 0ull, 0ull}; // rejected, hit, fallback, empty
    const BucketLayout& L = a.plan->L;
    for (uint32_t j = 0; j < kBkTile / kBkThreads; ++j) {
        const uint32_t i = base + j * kBkThreads + threadIdx.x;
        c += (uint32_t)__builtin_popcountll(__ballot(qt_splits(a, i, n)));
        if (a.acc && i < n) { // qt_level_stats' counting, restated
            const RangeAux ax = a.aux[i];
            const uint32_t b = a.classifier ? a.rkey[i] : 0u;
            if (ax.flags & kAuxEmpty) {
                v[3] += 1;
                v[0] += a.classifier ? a.nd : 0ull;
            } else {
                v[2] += (ax.flags & kAuxFallback) ? 1ull : 0ull;
                if (ax.flags & kAuxHit) {
                    v[1] += 1;
                    if (a.classifier)
                        v[0] += (unsigned long long)a.porig[ax.pos] - (ax.pos - L.dbeg[b]);
                } else if (a.classifier) {
                    v[0] += a.nd - L.dcnt[b];
                }
            }
        }
    }
    if (lane == 0)
        wc[wv] = c;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            v[k] += (unsigned long long)__shfl_xor((long long)v[k], o, 64);
        if (lane == 0)
            part[wv][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < kBkThreads / 64; ++w)
            t += wc[w];
        a.tcount[blockIdx.x] = t;
    }
    if (a.acc && threadIdx.x < 4) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < kBkThreads / 64; ++w)
            t += part[w][threadIdx.x];
        if (t)
            atomicAdd(&a.acc[(blockIdx.x % a.shards) * a.stride + threadIdx.x], t);
    }
}

__global__ void __launch_bounds__(kBkThreads) qt_split_emit(QtSplitArgs a)
{
    __shared__ uint32_t wcnt[kBkThreads / 64];
    __shared__ uint32_t run;
    const uint32_t n = min(a.plan->nr, a.nmax), leaf_base = a.plan->leaf_base;
    const uint32_t base = blockIdx.x * kBkTile, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    if (wv == 0) { // the splits of the tiles before this one, read from qt_split_count's per-tile counts
        uint32_t before = 0, total = 0;
        for (uint32_t t = lane; t < gridDim.x; t += 64) {
            const uint32_t ct = a.tcount[t];
            before += t < blockIdx.x ? ct : 0u;
            total += ct;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            before += (uint32_t)__shfl_xor((int)before, o, 64);
            total += (uint32_t)__shfl_xor((int)total, o, 64);
        }
        if (lane == 0) {
            run = before;
            if (blockIdx.x == 0) { // the next level's count and leaf base
                a.next->nr = 4 * total;
                a.next->leaf_base = leaf_base + n - total;
            }
        }
    }
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (uint32_t j = 0; j < kBkTile / kBkThreads; ++j) {
        const uint32_t i = base + j * kBkThreads + threadIdx.x;
        const bool sp = qt_splits(a, i, n);
        const unsigned long long m = __ballot(sp);
        if (lane == 0)
            wcnt[wv] = (uint32_t)__builtin_popcountll(m);
        __syncthreads();
        uint32_t o = run + (uint32_t)__builtin_popcountll(m & below); // splits before item i
        for (uint32_t w = 0; w < wv; ++w)
            o += wcnt[w];
        if (i < n) {
            if (sp) {
                const frac_grid_item r = a.ranges[i];
                const uint32_t h = r.w / 2;
                a.next_ranges[4 * o + 0] = frac_grid_item{r.x, r.y, h, h, -1};
                a.next_ranges[4 * o + 1] = frac_grid_item{r.x + h, r.y, h, h, -1};
                a.next_ranges[4 * o + 2] = frac_grid_item{r.x, r.y + h, h, h, -1};
                a.next_ranges[4 * o + 3] = frac_grid_item{r.x + h, r.y + h, h, h, -1};
            } else if (leaf_base + (i - o) < a.leaf_cap) {
                if (a.leaves32) {
                    a.leaves32[leaf_base + (i - o)] = qt_leaf_of(a.out[i], a.dcols);
                } else {
                    a.leaves[leaf_base + (i - o)] = a.out[i];
                }
            }
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (uint32_t w = 0; w < kBkThreads / 64; ++w)
                run += wcnt[w];
        __syncthreads();
    }
}

// The per-item maps of a planned level (fill_range_slots, fill_tile_pos and fill_rbucket restated, run
// by qt_plan's threads), and the run's resets: best_key (none yet), the direct form's zeroed rconst
// words (mfma_range_prep accumulates into them), the fallback count.
struct QtFillArgs {
    const uint32_t* rord;     // bucket-sorted range order
    const uint32_t* rkey;     // per range: its bucket
    uint32_t copies;          // T = 8 Fourier: slot s ≥ nblocks·32 is the flipped copy of s − nblocks·32
    uint32_t nthreads;        // the grid's bound: max(slots, tile rows, ranges)
    int32_t* slot_range;
    uint32_t* range_slot;
    int32_t* tile_pos;
    uint2* rbucket;
    uint32_t* rconst;         // zeroed per slot when not null (the direct form)
    unsigned long long* best_key;
    uint32_t* fb_count;
};

__device__ inline void qt_fill_item(const QtFillArgs& a, const BucketLayout& L, uint32_t nblocks, uint32_t ntiles,
                                    uint32_t nr, uint32_t i)
{
    const uint32_t nslots = nblocks * 32u;
    if (i < nslots * a.copies) {
        const uint32_t s = i % nslots, b = layout_bucket_of_slot(L, s), k = s - L.slot_first[b];
        int32_t r = -1;
        if (k < L.rcnt[b]) {
            r = (int32_t)a.rord[L.rbeg[b] + k];
            if (i < nslots)
                a.range_slot[r] = s;
        }
        a.slot_range[i] = r;
        if (a.rconst)
            a.rconst[i] = 0u;
    }
    if (i < ntiles * 32u) {
        const uint32_t tile = i >> 5;
        uint32_t b = 0;
        for (uint32_t k = 1; k < L.nb; ++k)
            b = tile >= L.tile_first[k] ? k : b;
        const uint32_t j = i - 32u * L.tile_first[b];
        a.tile_pos[i] = j < L.dcnt[b] ? (int32_t)(L.dbeg[b] + j) : -1;
    }
    if (i < nr) {
        const uint32_t b = a.rkey[i];
        a.rbucket[i] = make_uint2(L.dbeg[b], L.dbeg[b] + L.dcnt[b]);
        a.best_key[i] = ~0ull;
    }
    if (i == 0)
        *a.fb_count = 0u;
}

// The frame's result for the host in one write to pinned memory: the leaf count (the leaf base after the
// last level) and the counters summed over their shards — no copy command and no second round trip.
struct QtFrameSum {
    uint32_t leaves, pad_;
    unsigned long long acc[9];
};

__global__ void __launch_bounds__(64) qt_finish(const DevPlan* __restrict__ last, int ran,
                                                const unsigned long long* __restrict__ acc, uint32_t shards,
                                                uint32_t stride, QtFrameSum* __restrict__ dst)
{
    const uint32_t i = threadIdx.x;
    if (i < stride && i < 9) {
        unsigned long long t = 0;
        for (uint32_t k = 0; k < shards; ++k)
            t += acc[k * stride + i];
        dst->acc[i] = t;
    }
    if (i == 0)
        dst->leaves = ran ? last->leaf_base : 0u;
}

// ---- the device planner of a quadtree level (prepare()'s layout and work lists, restated) ----
// From the bucket bounds of the level's domains and ranges (bucket_bounds over the sorted keys)
// it lays out the MFMA engine's 32-slot range blocks and 32-row domain tiles per bucket, and writes
// the search's work items {first block, blocks, tile begin, tile end} — groups of `bpw` blocks of one
// bucket × splits of the bucket's tiles, splits = ⌈target · tiles / Σ groups·tiles⌉ capped at tiles / 4, in
// prepare()'s (copy, bucket, group, split) order — and the CSR map block → entries (work·bpw + k)
// the resolve kernels read.  Every count goes to the DevPlan; the launches that follow use
// worst-case grids.  The frame's counters get the level's total / eligible pairs and the MFMA
// flops the search issues.  Every block recomputes the (at most 7-bucket) header; block 0 writes it.
struct QtPlanArgs {
    DevPlan* plan;
    const uint32_t* dfirst;  // [kMaxBuckets + 1] first pool position per bucket (nullptr: one bucket)
    const uint32_t* rfirst;  // [kMaxBuckets + 1] first bucket-sorted range per bucket
    uint32_t nb;             // buckets: 7 with the classifier, 1 without
    uint32_t nd;             // domains of the level
    uint32_t nr_init;        // the first level: its range count (host-known); ~0u: plan->nr (qt_scatter)
    uint32_t bpw;            // range blocks per work item (search_dft 8, search_mfma 4, search_mfma16 mfma16_bpw(T))
    uint32_t target;         // target work items (workgroups)
    uint32_t copies;         // T = 8 Fourier: 2 (flipped copies), else 1
    uint32_t mfma_per_pair;  // MFMA 32x32x16 per (range block, domain tile) pair: flops accounting
    uint32_t nwork_cap, nent_cap, nblocks_cap, ntiles_cap; // buffer capacities
    uint4* work;
    uint32_t* blk_ptr;       // [nblocks·copies + 1]
    uint32_t* blk_ent;
    unsigned long long* acc; // frame counters: [5] total mappings, [6] eligible pairs, [7] flops, [8] overflow
    QtFillArgs fill;         // the per-item maps, filled by the same launch (from the header in LDS)
};

struct QtPlanHeader {
    BucketLayout L;
    uint32_t blk_first[kMaxBuckets], blk_count[kMaxBuckets], tile_count[kMaxBuckets], ns[kMaxBuckets];
    uint32_t wbase[2 * kMaxBuckets + 1]; // first work item of (copy, bucket), in that order
    uint32_t ebase[2 * kMaxBuckets + 1]; // first CSR entry of (copy, bucket)
    uint32_t nr, nblocks, ntiles, nwork, nent;
    bool ok;
};

// the header, 16 threads: thread t < 8 lays out bucket t, then thread t < 16 the (copy t / 8, bucket t % 8)
// entry; the prefix sums over the 8 buckets and 16 entries are one thread's (32-bit arithmetic throughout)
__device__ inline void qt_plan_header(const QtPlanArgs& a, QtPlanHeader& h, uint32_t t)
{
    constexpr uint32_t B = kMaxBuckets;
    __shared__ unsigned long long gtiles_s;
    BucketLayout& L = h.L;
    if (t < B) {
        const uint32_t nr = a.nr_init != ~0u ? a.nr_init : a.plan->nr;
        const bool in = t < a.nb;
        L.dbeg[t] = in ? (a.dfirst ? a.dfirst[t] : 0u) : 0u;
        L.dcnt[t] = in ? (a.dfirst ? a.dfirst[t + 1] - a.dfirst[t] : a.nd) : 0u;
        L.rbeg[t] = in ? (a.rfirst ? a.rfirst[t] : 0u) : 0u;
        L.rcnt[t] = in ? (a.rfirst ? min(a.rfirst[t + 1], nr) - min(a.rfirst[t], nr) : nr) : 0u;
        h.blk_count[t] = (L.rcnt[t] + 31) / 32;
        h.tile_count[t] = (L.dcnt[t] + 31) / 32;
        if (t == 0)
            h.nr = nr;
    }
    __syncthreads();
    if (t == 0) {
        L.nb = a.nb;
        L.VT = 1;
        uint32_t nbk = 0, nt = 0;
        unsigned long long gtiles = 0; // Σ groups × tiles
        for (uint32_t b = 0; b < B; ++b) {
            h.blk_first[b] = nbk;
            L.slot_first[b] = 32 * nbk;
            nbk += h.blk_count[b];
            L.tile_first[b] = nt;
            nt += h.tile_count[b];
            if (b < a.nb && h.tile_count[b])
                gtiles += (unsigned long long)((h.blk_count[b] + a.bpw - 1) / a.bpw * a.copies) * h.tile_count[b];
        }
        h.nblocks = nbk;
        h.ntiles = nt;
        gtiles_s = gtiles;
    }
    __syncthreads();
    uint32_t nw = 0, ne = 0;
    if (t < 2 * B) {
        const uint32_t cp = t / B, b = t % B, tc = h.tile_count[b], bc = cp < a.copies ? h.blk_count[b] : 0u;
        uint32_t ns = 0;
        if (b < a.nb && tc && bc) {
            // splits in proportion to the bucket's tiles (prepare()'s build_work): ⌈target·tc / Σ groups·tiles⌉
            const uint64_t gt = gtiles_s, tw = work_target(a.target, gt);
            const uint32_t sp = gt ? (uint32_t)((tw * tc + gt - 1) / gt) : 1u;
            ns = max(1u, min(sp, max(1u, tc / 4u))); // ≤ tc: every split holds at least one tile
        }
        if (cp == 0)
            h.ns[b] = ns;
        nw = (bc + a.bpw - 1) / a.bpw * ns;
        ne = bc * ns;
        h.wbase[t] = nw; // counts first, prefix below
        h.ebase[t] = ne;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t w = 0, e = 0;
        for (uint32_t q = 0; q < 2 * B; ++q) {
            const uint32_t cw = h.wbase[q], ce = h.ebase[q];
            h.wbase[q] = w;
            h.ebase[q] = e;
            w += cw;
            e += ce;
        }
        h.wbase[2 * B] = w;
        h.ebase[2 * B] = e;
        h.nwork = w;
        h.nent = e;
        h.ok = w <= a.nwork_cap && e <= a.nent_cap && h.nblocks <= a.nblocks_cap && h.ntiles <= a.ntiles_cap;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(256) qt_plan(QtPlanArgs a)
{
    __shared__ QtPlanHeader h;
    qt_plan_header(a, h, threadIdx.x);
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x, gs = gridDim.x * blockDim.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        DevPlan& p = *a.plan;
        p.L = h.L;
        p.nr = h.nr;
        if (a.nr_init != ~0u)
            p.leaf_base = 0;
        p.nblocks = h.ok ? h.nblocks : 0u;
        p.ntiles = h.ok ? h.ntiles : 0u;
        p.nwork = h.ok ? h.nwork : 0u;
        p.nslots = h.ok ? h.nblocks * 32u : 0u; // resolve_dft's slots: one wave takes both copies of a slot
        p.flip_slots = a.copies == 2 ? h.nblocks * 32u : 0u;
        uint64_t elig = 0, flops = 0;
        for (uint32_t b = 0; b < a.nb; ++b) {
            elig += (uint64_t)h.L.rcnt[b] * h.L.dcnt[b];
            flops += (uint64_t)h.blk_count[b] * h.tile_count[b] * a.copies * a.mfma_per_pair * 32768ull;
        }
        atomicAdd(&a.acc[5], (unsigned long long)a.nd * h.nr);
        atomicAdd(&a.acc[6], (unsigned long long)elig);
        atomicAdd(&a.acc[7], (unsigned long long)flops);
        if (!h.ok)
            atomicAdd(&a.acc[8], 1ull); // the host fails the frame (a bound was wrong: never expected)
    }
    if (!h.ok)
        return;
    // work items, in (copy, bucket, group, split) order
    for (uint32_t w = gt; w < h.nwork; w += gs) {
        uint32_t q = 0;
        while (q + 1 < 2 * (uint32_t)kMaxBuckets && h.wbase[q + 1] <= w)
            ++q;
        const uint32_t cp = q / kMaxBuckets, b = q % kMaxBuckets, ns = h.ns[b], loc = w - h.wbase[q];
        const uint32_t g = (loc / ns) * a.bpw, sp = loc % ns, tc = h.tile_count[b];
        const uint32_t bf = cp * h.nblocks + h.blk_first[b];
        const uint32_t t0 = h.L.tile_first[b] + tc * sp / ns; // tc · ns ≤ 2^13 · 2^13: 32 bits
        const uint32_t t1 = h.L.tile_first[b] + tc * (sp + 1) / ns;
        a.work[w] = make_uint4(bf + g, min(a.bpw, h.blk_count[b] - g), t0, t1);
    }
    // the CSR map: block (copy, bucket, k) holds one entry per split of its bucket
    const uint32_t nbt = h.nblocks * a.copies;
    for (uint32_t i = gt; i <= nbt; i += gs) {
        if (i == nbt) {
            a.blk_ptr[i] = h.nent;
            continue;
        }
        const uint32_t cp = i / h.nblocks, loc = i % h.nblocks;
        uint32_t b = 0;
        for (uint32_t k = 1; k < a.nb; ++k)
            b = loc >= h.blk_first[k] ? k : b;
        const uint32_t k = loc - h.blk_first[b], ns = h.ns[b], q = cp * kMaxBuckets + b;
        const uint32_t base = h.ebase[q] + k * ns;
        a.blk_ptr[i] = base;
        for (uint32_t sp = 0; sp < ns; ++sp)
            a.blk_ent[base + sp] = (h.wbase[q] + (k / a.bpw) * ns + sp) * a.bpw + k % a.bpw;
    }
    // the per-item maps, one item per thread of the grid (sized for fill.nthreads)
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.fill.nthreads)
        qt_fill_item(a.fill, h.L, h.nblocks, h.ntiles, h.nr, i);
}

// createUniformGrid(W, H, size, off) on the device (image/partition2.hpp:123-133, frac_uniform_grid2):
// the first quadtree level's ranges, kept on the device across frames like the domain grids
// (also the frame's reset of `nz` counters, in place of a memset launch)
__global__ void __launch_bounds__(256) qt_uniform_grid(uint32_t nx, uint32_t n, uint32_t size, uint32_t off,
                                                       frac_grid_item* __restrict__ out,
                                                       unsigned long long* __restrict__ zero = nullptr, uint32_t nz = 0)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = frac_grid_item{(i % nx) * off, (i / nx) * off, size, size, -1};
    if (i < nz)
        zero[i] = 0ull;
}

} // namespace fracenc
