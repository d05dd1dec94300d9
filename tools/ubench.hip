// ubench.hip — instruction-rate and exactness probes that decide the search design.
//  1. issue rate of v_dot2_u32_u16 / v_dot4_u32_u8 / v_fma_f32 (SGPR operand, 8 chains)
//  2. exactness of v_mfma_f32_32x32x16_f16 on the integer encoding used by the MFMA
//     engine: A = r−128 ∈ [−128,127], B = D4−510 ∈ [−510,510], C = 1.5·2^23, so every
//     partial sum stays in [2^23, 2^24) where fp32 has unit spacing.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench tools/ubench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef unsigned char uc4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

constexpr int ITERS = 4096;

__global__ void k_dot2(const unsigned* __restrict__ s, unsigned* out)
{
    unsigned a[8];
    for (int i = 0; i < 8; ++i)
        a[i] = threadIdx.x + i;
    const unsigned v = threadIdx.x * 0x00010001u;
    for (int it = 0; it < ITERS; ++it) {
        const unsigned sv = s[it & 63];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            a[i] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, sv), __builtin_bit_cast(us2, v + i), a[i], false);
    }
    unsigned r = 0;
    for (int i = 0; i < 8; ++i)
        r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_dot4(const unsigned* __restrict__ s, unsigned* out)
{
    unsigned a[8];
    for (int i = 0; i < 8; ++i)
        a[i] = threadIdx.x + i;
    const unsigned v = threadIdx.x * 0x01010101u;
    for (int it = 0; it < ITERS; ++it) {
        const unsigned sv = s[it & 63];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            a[i] = __builtin_amdgcn_udot4(sv, v + i, a[i], false);
    }
    unsigned r = 0;
    for (int i = 0; i < 8; ++i)
        r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma(const float* __restrict__ s, float* out)
{
    float a[8];
    for (int i = 0; i < 8; ++i)
        a[i] = threadIdx.x + i;
    const float v = threadIdx.x * 1e-3f;
    for (int it = 0; it < ITERS; ++it) {
        const float sv = s[it & 63];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            a[i] = __builtin_fmaf(sv, v + i, a[i]);
    }
    float r = 0;
    for (int i = 0; i < 8; ++i)
        r += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// one 32x32x64 tile per wave: A[32][64], B[64][32] f16, C init 1.5*2^23
__global__ void k_mfma_exact(const _Float16* A, const _Float16* B, float* C)
{
    const int lane = threadIdx.x;
    float16v acc;
    for (int i = 0; i < 16; ++i)
        acc[i] = 12582912.0f;
    for (int ks = 0; ks < 4; ++ks) {
        half8 a, b;
        for (int j = 0; j < 8; ++j) {
            const int k = ks * 16 + 8 * (lane >> 5) + j;
            a[j] = A[(lane & 31) * 64 + k];
            b[j] = B[k * 32 + (lane & 31)];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        C[row * 32 + (lane & 31)] = acc[i];
    }
}

__global__ void k_mfma_rate(float* out, int iters)
{
    half8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)(threadIdx.x + j);
        b[j] = (_Float16)(j - 3);
    }
    float16v acc0 = {}, acc1 = {};
    for (int it = 0; it < iters; ++it) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc1, 0, 0, 0);
    }
    float r = 0;
    for (int i = 0; i < 16; ++i)
        r += acc0[i] + acc1[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <class F>
double time_ms(F f)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < 5; ++i)
        f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5.0;
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 8, threads = 256;
    unsigned* s;
    unsigned* out;
    CK(hipMalloc(&s, 256 * 4));
    CK(hipMemset(s, 1, 256 * 4));
    CK(hipMalloc(&out, (size_t)blocks * threads * 4));
    const double instr = (double)blocks * (threads / 64) * ITERS * 8; // wave-instructions
    double ms = time_ms([&] { k_dot2<<<blocks, threads>>>(s, out); });
    printf("dot2_u32_u16: %.3f ms, %.1f Gwave-instr/s, %.1f cyc/instr/SIMD @2.4GHz, %.1f TOP/s (4 op/lane)\n", ms,
           instr / ms * 1e-6, cus * 4 * 2.4e9 / (instr / ms * 1e3), instr * 64 * 4 / ms * 1e-9);
    ms = time_ms([&] { k_dot4<<<blocks, threads>>>(s, out); });
    printf("dot4_u32_u8:  %.3f ms, %.1f Gwave-instr/s, %.1f cyc/instr/SIMD, %.1f TOP/s (8 op/lane)\n", ms,
           instr / ms * 1e-6, cus * 4 * 2.4e9 / (instr / ms * 1e3), instr * 64 * 8 / ms * 1e-9);
    ms = time_ms([&] { k_fma<<<blocks, threads>>>((const float*)s, (float*)out); });
    printf("fma_f32:      %.3f ms, %.1f Gwave-instr/s, %.1f cyc/instr/SIMD, %.1f TFLOP/s\n", ms, instr / ms * 1e-6,
           cus * 4 * 2.4e9 / (instr / ms * 1e3), instr * 64 * 2 / ms * 1e-9);
    const int miters = 2048;
    float* fo;
    CK(hipMalloc(&fo, (size_t)blocks * threads * 4));
    ms = time_ms([&] { k_mfma_rate<<<blocks, threads>>>(fo, miters); });
    const double flops = (double)blocks * (threads / 64) * miters * 2 * 32 * 32 * 16 * 2;
    printf("mfma_f32_32x32x16_f16: %.3f ms, %.1f TFLOP/s\n", ms, flops / ms * 1e-9);

    // exactness
    std::mt19937 rng(1);
    _Float16 *dA, *dB;
    float* dC;
    CK(hipMalloc(&dA, 32 * 64 * 2));
    CK(hipMalloc(&dB, 64 * 32 * 2));
    CK(hipMalloc(&dC, 32 * 32 * 4));
    std::vector<_Float16> A(32 * 64), B(64 * 32);
    std::vector<int> Ai(32 * 64), Bi(64 * 32);
    std::vector<float> Cg(32 * 32);
    long bad = 0, total = 0;
    for (int trial = 0; trial < 400; ++trial) {
        for (int i = 0; i < 32 * 64; ++i) {
            int a = (int)(rng() % 256) - 128, b = (int)(rng() % 1021) - 510;
            if (trial % 4 == 1) {
                a = (rng() & 1) ? 127 : -128;
                b = (rng() & 1) ? 510 : -510;
            } else if (trial % 4 == 2) {
                a = -128;
                b = (i % 2) ? 510 : -510;
            } else if (trial % 4 == 3) {
                a = (i % 3) - 1;
                b = (int)(rng() % 3) - 1;
            }
            Ai[i] = a;
            Bi[i] = b;
            A[i] = (_Float16)a;
            B[i] = (_Float16)b;
        }
        CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice));
        k_mfma_exact<<<1, 64>>>(dA, dB, dC);
        CK(hipMemcpy(Cg.data(), dC, Cg.size() * 4, hipMemcpyDeviceToHost));
        for (int r = 0; r < 32; ++r)
            for (int c = 0; c < 32; ++c) {
                long ref = 12582912;
                for (int k = 0; k < 64; ++k)
                    ref += (long)Ai[r * 64 + k] * Bi[k * 32 + c];
                ++total;
                if ((double)Cg[r * 32 + c] != (double)ref)
                    ++bad;
            }
    }
    printf("mfma f16 integer exactness: %ld / %ld mismatches\n", bad, total);
    return bad ? 1 : 0;
}
