// fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE on the search kernel's own access pattern
// (MI355X_MICROARCH.md §HBM: "calibrate on a known byte count in your own access pattern before
// trusting an absolute").  The Fourier search (fracenc_dft.hip search_dft, variant 35) stages domain
// tiles with buffer_load_dwordx4 … lds: per wave-instruction 1 KiB contiguous (16 B per lane), into a
// double-buffered LDS stage of 21 KiB, 8 waves per 512-thread workgroup, 2 workgroups per CU.
//
// Modes (one kernel each, same staging loop, a paced spin per stage in place of the MFMAs):
//   once   G workgroups, workgroup g streams its own CH-byte chunk once: the bytes read are known
//          exactly (G·CH), so FETCH_SIZE ÷ bytes is the counter's factor for this pattern;
//   shared G workgroups all stream the same S bytes from the start — the search's domain split read
//          by every workgroup of the split: FETCH_SIZE ÷ S counts the L2-miss passes over it.
// usage: fetch_calib once|shared BYTES WORKGROUPS SPIN_CYCLES
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

constexpr unsigned kWaves = 8, kStage = 21; // 21 KiB pieces of 1 KiB per stage, as search_dft

__global__ void __launch_bounds__(64 * kWaves) stream_lds(const uint4* src, size_t chunk, int shared, unsigned spin,
                                                          unsigned* sink)
{
    __shared__ uint4 lds[2][kStage * 64];
    const size_t base = shared ? 0 : (size_t)blockIdx.x * chunk;
    const unsigned wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned voff = (threadIdx.x & 63u) * 16u;
    const size_t pieces = chunk / 1024, nst = (pieces + kStage - 1) / kStage;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)src + base), 0, 0xffffffffu,
                                                                  0x00020000);
    unsigned acc = 0;
    auto stage = [&](int b, size_t st) {
        const size_t p0 = st * kStage;
        for (unsigned p = wv; p < kStage && p0 + p < pieces; p += kWaves)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds[b] + p * 64),
                                                     16, voff, (unsigned)((p0 + p) * 1024), 0, 0);
    };
    if (nst)
        stage(0, 0);
    for (size_t st = 0; st < nst; ++st) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (st + 1 < nst)
            stage((int)((st + 1) & 1), st + 1);
        acc += lds[st & 1][threadIdx.x].x;
        // paced in place of the search's MFMAs: the workgroups drift as the search's do
        const long long t0 = clock64();
        while (clock64() - t0 < (long long)spin)
            ;
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

int main(int argc, char** argv)
{
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s once|shared BYTES WORKGROUPS SPIN_CYCLES\n", argv[0]);
        return 2;
    }
    const int shared = std::strcmp(argv[1], "shared") == 0;
    const size_t bytes = std::strtoull(argv[2], nullptr, 10) / 1024 * 1024;
    const unsigned G = (unsigned)std::atoi(argv[3]), spin = (unsigned)std::atoi(argv[4]);
    const size_t chunk = shared ? bytes : bytes / G / 1024 * 1024;
    const size_t alloc = shared ? bytes : chunk * G;
    uint4* src = nullptr;
    unsigned* sink = nullptr;
    if (hipMalloc(&src, alloc + 65536) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess)
        return 1;
    hipMemset(src, 1, alloc);
    for (int rep = 0; rep < 3; ++rep)
        stream_lds<<<G, 64 * kWaves>>>(src, chunk, shared, spin, sink);
    if (hipDeviceSynchronize() != hipSuccess)
        return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    stream_lds<<<G, 64 * kWaves>>>(src, chunk, shared, spin, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::printf("{\"mode\": \"%s\", \"workgroups\": %u, \"chunk_bytes\": %zu, \"bytes_read_per_launch\": %zu, "
                "\"distinct_bytes\": %zu, \"spin\": %u, \"ms\": %.4f}\n",
                argv[1], G, chunk, chunk * G, alloc, spin, ms);
    hipFree(src);
    hipFree(sink);
    return 0;
}
