// Standalone probe of the classifier's block-sum path (fracenc_bucket.hip frame_block_sums + bucket_keys_bs)
// against a host computation: the pyramid levels, and the categories of the quadtree's grids, on a random
// plane whose sides are not multiples of 16.  Also an unaligned 32-bit load from a u16 array.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I fractencode_amd/csrc tools/bsum_probe.hip -o tools/_bsum_probe
#include "fracenc_classify.hip"
#include "fracenc_bucket.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace fracenc;

static int cat_host(uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4)
{
    static const unsigned char rules[24][4] = {
        {1, 2, 3, 4}, {3, 1, 4, 2}, {4, 3, 2, 1}, {2, 4, 1, 3}, {1, 3, 2, 4}, {2, 1, 4, 3},
        {4, 2, 3, 1}, {3, 4, 1, 2}, {1, 4, 3, 2}, {4, 1, 2, 3}, {3, 2, 4, 1}, {2, 3, 1, 4},
        {1, 2, 4, 3}, {3, 1, 2, 4}, {4, 3, 1, 2}, {2, 4, 3, 1}, {2, 1, 3, 4}, {1, 3, 4, 2},
        {3, 4, 2, 1}, {4, 2, 1, 3}, {1, 4, 2, 3}, {4, 1, 3, 4}, {2, 3, 4, 1}, {3, 2, 1, 4},
    };
    const uint32_t a[5] = {0u, a1, a2, a3, a4};
    for (int r = 0; r < 24; ++r)
        if (a[rules[r][0]] > a[rules[r][1]] && a[rules[r][1]] > a[rules[r][2]] && a[rules[r][2]] > a[rules[r][3]])
            return r / 4;
    return -1;
}

__global__ void unaligned_probe(const uint16_t* p, uint32_t* out)
{
    out[threadIdx.x] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(p) + 2 + 4 * threadIdx.x);
}

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                                     \
            return 2;                                                                                                  \
        }                                                                                                              \
    } while (0)

int main()
{
    int bad = 0;
    { // unaligned 32-bit load
        std::vector<uint16_t> h(130);
        for (int i = 0; i < 130; ++i)
            h[i] = (uint16_t)(1000 + i);
        uint16_t* d;
        uint32_t* o;
        CK(hipMalloc(&d, 130 * 2));
        CK(hipMalloc(&o, 64 * 4));
        CK(hipMemcpy(d, h.data(), 260, hipMemcpyHostToDevice));
        unaligned_probe<<<1, 64>>>(d, o);
        std::vector<uint32_t> r(64);
        CK(hipMemcpy(r.data(), o, 256, hipMemcpyDeviceToHost));
        int wrong = 0;
        for (int t = 0; t < 64; ++t)
            wrong += r[t] != ((uint32_t)h[1 + 2 * t] | ((uint32_t)h[2 + 2 * t] << 16));
        std::printf("unaligned dword loads wrong: %d / 64 (first: got %08x want %08x)\n", wrong, r[0],
                    (uint32_t)h[1] | ((uint32_t)h[2] << 16));
        hipFree(d);
        hipFree(o);
    }
    const uint32_t W = 2050, H = 2046, stride = 2112;
    std::vector<uint8_t> plane((size_t)stride * H);
    uint32_t s = 12345;
    for (auto& v : plane) {
        s = s * 1664525u + 1013904223u;
        v = (uint8_t)(s >> 24);
    }
    uint8_t* dp;
    uint16_t* db;
    CK(hipMalloc(&dp, plane.size()));
    CK(hipMemcpy(dp, plane.data(), plane.size(), hipMemcpyHostToDevice));
    const size_t nw = bs_words(W, H);
    CK(hipMalloc(&db, nw * 2));
    CK(hipMemset(db, 0xff, nw * 2));
    launch_block_sums(dp, stride, W, H, db, 0);
    CK(hipDeviceSynchronize());
    std::vector<uint16_t> hb(nw);
    CK(hipMemcpy(hb.data(), db, nw * 2, hipMemcpyDeviceToHost));
    const BlockSums b = bs_layout(db, W, H);
    for (int l = 0; l < 4; ++l) {
        const uint32_t q = 2u << l;
        int wrong = 0;
        for (uint32_t y = 0; y < b.rows[l]; ++y)
            for (uint32_t x = 0; x < b.cols[l]; ++x) {
                uint32_t t = 0;
                for (uint32_t i = 0; i < q; ++i)
                    for (uint32_t j = 0; j < q; ++j)
                        t += plane[(size_t)(y * q + i) * stride + x * q + j];
                const uint16_t got = hb[(b.s[l] - db) + (size_t)y * b.pitch[l] + x];
                if (got != t && wrong++ < 3)
                    std::printf("level q=%u (%u,%u): got %u want %u\n", q, x, y, got, t);
            }
        std::printf("pyramid q=%u: %d wrong of %u\n", q, wrong, b.rows[l] * b.cols[l]);
        bad += wrong;
    }
    // categories of uniform grids 2n at stride n (domains) and n at stride n (ranges), n = 16, 8, 4, 2; at
    // n = 4 also 8×8 at stride 2 (half the items off the level's alignment) and 6×6 at stride 3 (no level):
    // the per-thread pixel sums
    for (uint32_t n = 16; n >= 2; n /= 2) {
        for (int kind = 0; kind < (n == 4 ? 4 : 2); ++kind) {
            const uint32_t sz = kind == 3 ? 6 : kind == 1 ? n : 2 * n, st = kind == 2 ? 2 : kind == 3 ? 3 : n;
            std::vector<frac_grid_item> items;
            for (uint32_t y = 0; y + sz <= H; y += st)
                for (uint32_t x = 0; x + sz <= W; x += st)
                    items.push_back(frac_grid_item{x, y, sz, sz, -1});
            frac_grid_item* di;
            uint32_t* dk;
            CK(hipMalloc(&di, items.size() * sizeof(frac_grid_item)));
            CK(hipMalloc(&dk, items.size() * 4));
            CK(hipMemcpy(di, items.data(), items.size() * sizeof(frac_grid_item), hipMemcpyHostToDevice));
            KeySeg k0{di, (uint32_t)items.size(), dp, stride, dk, nullptr, nullptr, nullptr};
            KeySeg k1{di, 0u, dp, stride, dk, nullptr, nullptr, nullptr};
            launch_bucket_keys_bs(k0, b, sz, sz, k1, b, sz, sz, 0);
            CK(hipDeviceSynchronize());
            std::vector<uint32_t> hk(items.size());
            CK(hipMemcpy(hk.data(), dk, hk.size() * 4, hipMemcpyDeviceToHost));
            int wrong = 0;
            for (size_t i = 0; i < items.size(); ++i) {
                const frac_grid_item& it = items[i];
                const uint32_t hw = it.w / 2;
                uint32_t qq[4] = {0, 0, 0, 0};
                for (uint32_t py = 0; py < it.h; ++py)
                    for (uint32_t px = 0; px < it.w; ++px)
                        qq[(py >= hw ? 2 : 0) + (px >= hw ? 1 : 0)] += plane[(size_t)(it.y + py) * stride + it.x + px];
                const uint32_t want = (uint32_t)(cat_host(qq[0] & 0xffff, qq[1] & 0xffff, qq[2] & 0xffff, qq[3] & 0xffff) + 1);
                if (hk[i] != want && wrong++ < 3)
                    std::printf("n=%u kind %d (%u,%u): key %u want %u\n", n, kind, it.x, it.y, hk[i], want);
            }
            std::printf("keys n=%u kind %d (%ux%u stride %u): %d wrong of %zu\n", n, kind, sz, sz, st, wrong, items.size());
            bad += wrong;
            hipFree(di);
            hipFree(dk);
        }
    }
    std::printf(bad ? "FAIL\n" : "OK\n");
    return bad ? 1 : 0;
}
