// fracenc_classify.hip — the classifier pre-pass on the device
// (BrightnessBlocksClassifier2::getCategory, encode/Classifier2.cpp:8-62, preclassify :64-68).
//
// One wave per grid item: lanes stride over the item's pixels, accumulating the four
// quadrant sums (GridItemBase::topLeft … bottomRight, image/partition2.hpp:13-31, each
// size/2); ImageStatistics2::sum keeps u16 arithmetic for quadrants up to 16 wide
// (image/ImageStatistics.cpp:4-51), so those sums are taken mod 2^16.  The 24 strict-order
// rules then give the category 0..5 or −1 (the rule at Classifier2.cpp:48 is contradictory
// and never fires).  The sums are exact integers, so comparing them as integers is
// comparing the reference's doubles.
#include "fracenc_common.h"

namespace fracenc {

__device__ inline int category4_dev(uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4)
{
    // quadruples (i j k l): a_i > a_j > a_k > a_l, in the reference's order, 4 rules per category
    constexpr unsigned char rules[24][4] = {
        {1, 2, 3, 4}, {3, 1, 4, 2}, {4, 3, 2, 1}, {2, 4, 1, 3}, {1, 3, 2, 4}, {2, 1, 4, 3},
        {4, 2, 3, 1}, {3, 4, 1, 2}, {1, 4, 3, 2}, {4, 1, 2, 3}, {3, 2, 4, 1}, {2, 3, 1, 4},
        {1, 2, 4, 3}, {3, 1, 2, 4}, {4, 3, 1, 2}, {2, 4, 3, 1}, {2, 1, 3, 4}, {1, 3, 4, 2},
        {3, 4, 2, 1}, {4, 2, 1, 3}, {1, 4, 2, 3}, {4, 1, 3, 4}, {2, 3, 4, 1}, {3, 2, 1, 4},
    };
    const uint32_t a[5] = {0u, a1, a2, a3, a4};
#pragma unroll
    for (int r = 0; r < 24; ++r)
        if (a[rules[r][0]] > a[rules[r][1]] && a[rules[r][1]] > a[rules[r][2]] && a[rules[r][2]] > a[rules[r][3]])
            return r / 4;
    return -1;
}

struct ClassifyArgs {
    const uint8_t* plane;
    uint32_t stride;
    const frac_grid_item* items;
    const uint32_t* list; // indices into items (nullptr: items 0..n-1)
    uint32_t n;
    int32_t* out;         // category per list entry
};

__global__ void __launch_bounds__(256) classify_items(ClassifyArgs a)
{
    const uint32_t k = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (k >= a.n)
        return;
    const frac_grid_item it = a.items[a.list ? a.list[k] : k];
    const uint32_t hw = it.w / 2, hh = it.h / 2;
    uint32_t q[4] = {0u, 0u, 0u, 0u};
    // quadrant (qx, qy) covers [x + qx·hw, +hw) × [y + qy·hh, +hh); an odd size leaves the
    // last column / row outside every quadrant, as in the reference
    const uint32_t qw = 2 * hw, npx = qw * (2 * hh);
    for (uint32_t p = lane; p < npx; p += 64) {
        const uint32_t px = p % qw, py = p / qw;
        const uint32_t v = a.plane[(size_t)(it.y + py) * a.stride + it.x + px];
        q[(py >= hh ? 2 : 0) + (px >= hw ? 1 : 0)] += v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            q[i] += (uint32_t)__shfl_xor((int)q[i], o, 64);
    if (lane == 0) {
        if (hw <= 16)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                q[i] &= 0xffffu;
        a.out[k] = category4_dev(q[0], q[1], q[2], q[3]);
    }
}

} // namespace fracenc
