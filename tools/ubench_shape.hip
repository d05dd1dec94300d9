// ubench_shape.hip — the search's tile loop in two MFMA shapes, on LDS-resident random integer
// operands of the search's magnitudes (no DMA, no guard, no chunk bookkeeping):
//   k32: the shipped six-MFMA form, v_mfma_f32_32x32x16_f16, 32 ranges × 32 domains per tile pair,
//        A fragments (5) and row constants (16 per lane) from LDS, B fragments (6) in registers;
//   k16: a four-MFMA form of the same candidate values in v_mfma_f32_16x16x32_f16 (K = 32 holds both
//        halves of a bin: 2U = [B0|B2]·[A0;A2], 2U' = [B0|B2]·[A0;−A2], 2Pr = [γ|δ]·[2α;2β],
//        2Pi = [γ|δ]·[2β;−2α]), 16 ranges × 16 domains per tile pair, ≈50 VGPRs (8 waves/SIMD).
// k16 issues 4/3 of k32's matrix work per (range, domain) pair; the question is whether its
// occupancy and shape recover that.  Prints (range, domain) pairs per second for each.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_shape tools/ubench_shape.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e = (x);                                                                                            \
        if (e != hipSuccess) {                                                                                         \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                                            \
            exit(2);                                                                                                   \
        }                                                                                                              \
    } while (0)

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int NT = 8; // 32-domain tiles resident in LDS

// k32: LDS = NT × (5 A pieces of 1 KiB) + NT × 16 uint4 of constants
// F5: the five-MFMA form with the folded constant (P from C = −Σb²/2, M separate; 2U − Σb²/2 = P + M and
// 2U' − Σb²/2 = P − M on the VALU): 5 MFMA and 5 VALU per candidate instead of 6 and 3
template <int WPE, bool F5 = false>
__global__ void __launch_bounds__(512, WPE) k32(const uint4* __restrict__ src, const uint4* __restrict__ rf, int iters,
                                              float* out)
{
    constexpr int A = NT * 5 * 64, C = NT * 16;
    __shared__ uint4 lds[A + C];
    for (int i = threadIdx.x; i < A + C; i += 512)
        lds[i] = src[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5;
    half8 bf[6];
    for (int f = 0; f < 6; ++f)
        bf[f] = __builtin_bit_cast(half8, rf[((blockIdx.x * 8 + (threadIdx.x >> 6)) % 64 * 6 + f) * 64 + lane]);
    float m = -__builtin_inff();
    for (int it = 0; it < iters; ++it) {
#pragma unroll 2
        for (int q = 0; q < NT; ++q) {
            half8 af[5];
#pragma unroll
            for (int s = 0; s < 5; ++s)
                af[s] = __builtin_bit_cast(half8, lds[(q * 5 + s) * 64 + lane]);
            f16v c;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = lds[A + q * 16 + h * 4 + k];
                c[4 * k] = __uint_as_float(v.x);
                c[4 * k + 1] = __uint_as_float(v.y);
                c[4 * k + 2] = __uint_as_float(v.z);
                c[4 * k + 3] = __uint_as_float(v.w);
            }
            const f16v z = {};
            const f16v k1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bf[3], z, 0, 0, 0);
            const f16v p = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[0], c, 0, 0, 0);
            const f16v pr = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bf[4], k1, 0, 0, 0);
            if constexpr (F5) {
                const f16v mm = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[1], z, 0, 0, 0);
                const f16v pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], bf[5], k1, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    m = __builtin_fmaxf(__builtin_fmaxf(m, (p[i] + mm[i]) + __builtin_fabsf(pr[i])),
                                        (p[i] - mm[i]) + __builtin_fabsf(pi[i]));
            } else {
                const f16v u = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[1], p, 0, 0, 0);
                const f16v pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], bf[5], k1, 0, 0, 0);
                const f16v v = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[2], p, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    m = __builtin_fmaxf(__builtin_fmaxf(m, u[i] + __builtin_fabsf(pr[i])), v[i] + __builtin_fabsf(pi[i]));
            }
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = m;
}

// k16: LDS = NT × 2 sub-tiles × (2 A pieces of 1 KiB) + NT × 2 × 4 uint4 of constants (4 rows per lane group)
template <int WPE>
__global__ void __launch_bounds__(512, WPE) k16(const uint4* __restrict__ src, const uint4* __restrict__ rf, int iters,
                                                 float* out)
{
    constexpr int A = NT * 2 * 2 * 64, C = NT * 2 * 4;
    __shared__ uint4 lds[A + C];
    for (int i = threadIdx.x; i < A + C; i += 512)
        lds[i] = src[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane >> 4;
    half8 bf[4];
    for (int f = 0; f < 4; ++f)
        bf[f] = __builtin_bit_cast(half8, rf[((blockIdx.x * 8 + (threadIdx.x >> 6)) % 64 * 6 + f) * 64 + lane]);
    float m = -__builtin_inff();
    for (int it = 0; it < iters; ++it) {
#pragma unroll 4
        for (int q = 0; q < 2 * NT; ++q) {
            const half8 a0 = __builtin_bit_cast(half8, lds[(q * 2) * 64 + lane]);
            const half8 a1 = __builtin_bit_cast(half8, lds[(q * 2 + 1) * 64 + lane]);
            const uint4 cv = lds[A + q * 4 + g];
            const f4v c = {__uint_as_float(cv.x), __uint_as_float(cv.y), __uint_as_float(cv.z), __uint_as_float(cv.w)};
            const f4v z = {};
            const f4v u = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bf[0], c, 0, 0, 0);
            const f4v v = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bf[1], c, 0, 0, 0);
            const f4v pr = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bf[2], z, 0, 0, 0);
            const f4v pi = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bf[3], z, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                m = __builtin_fmaxf(__builtin_fmaxf(m, u[i] + __builtin_fabsf(pr[i])), v[i] + __builtin_fabsf(pi[i]));
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = m;
}

// kl: the six-MFMA loop with five B fragments (the negated one moved to the domain side: 2U' = P − M from
// a sixth A fragment −(s_b − u_b) against s_a − u_a), WAVES waves per workgroup, at least WPE waves per SIMD
// (10-wave workgroups at WPE 5: 20 waves per CU = 5 per SIMD)
template <int WAVES, int WPE>
__global__ void __launch_bounds__(64 * WAVES, WPE) kl(const uint4* __restrict__ src, const uint4* __restrict__ rf,
                                                       int iters, float* out)
{
    constexpr int A = NT * 6 * 64, C = NT * 16;
    __shared__ uint4 lds[A + C];
    for (int i = threadIdx.x; i < A + C; i += 64 * WAVES)
        lds[i] = src[i % (NT * 5 * 64 + NT * 16)];
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5;
    half8 bf[5];
    for (int f = 0; f < 5; ++f)
        bf[f] = __builtin_bit_cast(half8, rf[((blockIdx.x * WAVES + (threadIdx.x >> 6)) % 64 * 6 + f) * 64 + lane]);
    float m = -__builtin_inff();
    for (int it = 0; it < iters; ++it) {
#pragma unroll 1
        for (int q = 0; q < NT; ++q) {
            half8 af[6];
#pragma unroll
            for (int s = 0; s < 6; ++s)
                af[s] = __builtin_bit_cast(half8, lds[(q * 6 + s) * 64 + lane]);
            f16v c;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = lds[A + q * 16 + h * 4 + k];
                c[4 * k] = __uint_as_float(v.x);
                c[4 * k + 1] = __uint_as_float(v.y);
                c[4 * k + 2] = __uint_as_float(v.z);
                c[4 * k + 3] = __uint_as_float(v.w);
            }
            const f16v z = {};
            const f16v k1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[2], bf[2], z, 0, 0, 0);
            const f16v p = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[0], c, 0, 0, 0);
            const f16v pr = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[3], bf[3], k1, 0, 0, 0);
            const f16v u = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[1], p, 0, 0, 0);
            const f16v pi = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[4], bf[4], k1, 0, 0, 0);
            const f16v v = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[5], bf[1], p, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i)
                m = __builtin_fmaxf(__builtin_fmaxf(m, u[i] + __builtin_fabsf(pr[i])), v[i] + __builtin_fabsf(pi[i]));
        }
    }
    out[blockIdx.x * 64 * WAVES + threadIdx.x] = m;
}

static uint4 rand_frag(std::mt19937& g, int lo, int hi)
{
    std::uniform_int_distribution<int> d(lo, hi);
    _Float16 h[8];
    for (int i = 0; i < 8; ++i)
        h[i] = (_Float16)d(g);
    uint4 r;
    memcpy(&r, h, 16);
    return r;
}

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const int nwg = argc > 2 ? atoi(argv[2]) : 4096;
    std::mt19937 g(7);
    // the search's operand magnitudes: domain fragments |·| ≤ 2048 (typ. a few hundred), range ≤ 512
    const int na = NT * 5 * 64 + NT * 16;
    std::vector<uint4> hs(na), hr(64 * 6 * 64);
    for (int i = 0; i < NT * 5 * 64; ++i)
        hs[i] = rand_frag(g, -400, 400);
    std::uniform_int_distribution<int> dc(-200000, -1000);
    for (int i = NT * 5 * 64; i < na; ++i) {
        const float f[4] = {(float)dc(g), (float)dc(g), (float)dc(g), (float)dc(g)};
        memcpy(&hs[i], f, 16);
    }
    for (auto& x : hr)
        x = rand_frag(g, -120, 120);
    const int a16 = NT * 2 * 2 * 64, n16 = a16 + NT * 2 * 4;
    std::vector<uint4> h16(n16);
    for (int i = 0; i < a16; ++i)
        h16[i] = rand_frag(g, -400, 400);
    for (int i = a16; i < n16; ++i) {
        const float f[4] = {(float)dc(g), (float)dc(g), (float)dc(g), (float)dc(g)};
        memcpy(&h16[i], f, 16);
    }
    uint4 *ds, *dr, *d16;
    float* dout;
    CK(hipMalloc(&d16, h16.size() * 16));
    CK(hipMemcpy(d16, h16.data(), h16.size() * 16, hipMemcpyHostToDevice));
    CK(hipMalloc(&ds, hs.size() * 16));
    CK(hipMalloc(&dr, hr.size() * 16));
    CK(hipMalloc(&dout, (size_t)nwg * 512 * 4));
    CK(hipMemcpy(ds, hs.data(), hs.size() * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, hr.data(), hr.size() * 16, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch, double pairs) {
        for (int w = 0; w < 3; ++w)
            launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-10s %8.3f ms  %.3e pairs/s\n", name, best, pairs / (best * 1e-3));
        fflush(stdout);
    };
    // pairs per launch: waves × iters × NT tiles × (32×32 | 16×16·2) pairs
    const double waves = (double)nwg * 8;
    run("k32", [&]() { k32<4><<<nwg, 512>>>(ds, dr, iters, dout); }, waves * iters * NT * 1024.0);
    run("k32/w5", [&]() { k32<5><<<nwg, 512>>>(ds, dr, iters, dout); }, waves * iters * NT * 1024.0);
    run("k32/w3", [&]() { k32<3><<<nwg, 512>>>(ds, dr, iters, dout); }, waves * iters * NT * 1024.0);
    run("k32f5", [&]() { k32<4, true><<<nwg, 512>>>(ds, dr, iters, dout); }, waves * iters * NT * 1024.0);
    run("kl8/w4", [&]() { kl<8, 4><<<nwg, 512>>>(ds, dr, iters, dout); }, waves * iters * NT * 1024.0);
    {
        const int nwg10 = nwg * 8 / 10; // the same waves in 10-wave workgroups
        run("kl10/w5", [&]() { kl<10, 5><<<nwg10, 640>>>(ds, dr, iters, dout); }, (double)nwg10 * 10 * iters * NT * 1024.0);
    }
    run("k16/w8", [&]() { k16<8><<<nwg, 512>>>(d16, dr, iters, dout); }, waves * iters * NT * 512.0);
    run("k16/w4", [&]() { k16<4><<<nwg, 512>>>(d16, dr, iters, dout); }, waves * iters * NT * 512.0);
    run("k32", [&]() { k32<4><<<nwg, 512>>>(ds, dr, iters, dout); }, waves * iters * NT * 1024.0);
    return 0;
}
