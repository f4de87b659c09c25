// Micro-benchmarks of the access patterns the Plumtree round kernel uses.
// hipcc --offload-arch=gfx950 -O3 -o /tmp/mb tools/microbench.hip && /tmp/mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void scatter32(uint32_t* __restrict__ out, const uint32_t* __restrict__ idx, uint32_t m) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[idx[i]] = i | 1u;
}
__global__ void scatter8(uint8_t* __restrict__ out, const uint32_t* __restrict__ idx, uint32_t m, uint32_t mask) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[idx[i] & mask] = 1;
}
__global__ void scatter16(uint16_t* __restrict__ out, const uint32_t* __restrict__ idx, uint32_t m, uint32_t mod) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[idx[i] % mod] = (uint16_t)i;
}
__global__ void scatter8m(uint8_t* __restrict__ out, const uint32_t* __restrict__ idx, uint32_t m, uint32_t mod) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[idx[i] % mod] = (uint8_t)i;
}
__global__ void gather128(uint4* __restrict__ out, const uint4* __restrict__ in, const uint32_t* __restrict__ idx, uint32_t m, uint32_t mod) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[i & 1023] = in[idx[i] % mod];
}
__global__ void gather32(uint32_t* __restrict__ out, const uint32_t* __restrict__ in, const uint32_t* __restrict__ idx, uint32_t m) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[i] = in[idx[i]];
}
__global__ void copy128(uint4* __restrict__ out, const uint4* __restrict__ in, uint32_t m) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[i] = in[i];
}
__global__ void scan8(const uint8_t* __restrict__ in, uint32_t n, uint32_t* cnt) {
    uint32_t c = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) c += in[i];
    if (c) atomicAdd(cnt, c);
}
__global__ void scan128(const uint4* __restrict__ in, uint32_t n16, uint32_t* cnt) {
    uint32_t c = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) {
        uint4 x = in[i]; c += (x.x | x.y | x.z | x.w) != 0;
    }
    if (c) atomicAdd(cnt, c);
}
__global__ void empty_kernel() {}
// a round kernel's idle workgroup: read the chunk's 64 group flags (1 load), barrier, exit
__global__ __launch_bounds__(256) void idle_chunks(const uint8_t* __restrict__ pend, uint32_t* cnt) {
    extern __shared__ uint32_t lds[];
    __shared__ uint32_t any;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    if (threadIdx.x < 64 && pend[blockIdx.x * 64 + threadIdx.x]) atomicOr(&any, 1u);
    __syncthreads();
    if (any) { lds[threadIdx.x] = any; __syncthreads(); if (threadIdx.x == 0) atomicAdd(cnt, lds[1]); }
}
// the same with a chain of three dependent loads before the flags (counts, scalar, flags)
__global__ __launch_bounds__(256) void idle_chain(const uint8_t* __restrict__ pend, const uint32_t* c3, uint32_t* cnt) {
    __shared__ uint32_t any, k;
    if (threadIdx.x == 0) { any = 0; k = c3[blockIdx.x & 63]; }
    __syncthreads();
    const uint32_t kk = c3[64 + (k & 63)];
    if (threadIdx.x < 64 && pend[blockIdx.x * 64 + threadIdx.x + (kk & 1)]) atomicOr(&any, 1u);
    __syncthreads();
    if (any && threadIdx.x == 0) atomicAdd(cnt, 1u);
}

int main() {
    const uint32_t E = 50'000'000, M = 26'000'000, N = 10'000'000;
    std::vector<uint32_t> h(M);
    std::mt19937 rng(1);
    for (auto& x : h) x = rng() % E;
    uint32_t *idx, *buf, *out, *cnt; uint8_t* flags;
    CK(hipMalloc(&idx, M * 4)); CK(hipMalloc(&buf, E * 4ull)); CK(hipMalloc(&out, E * 4ull));
    CK(hipMalloc(&flags, N)); CK(hipMalloc(&cnt, 4));
    CK(hipMemcpy(idx, h.data(), M * 4, hipMemcpyHostToDevice));
    CK(hipMemset(buf, 0, E * 4ull)); CK(hipMemset(flags, 0, N));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto T = [&](const char* name, double bytes, auto fn) {
        for (int w = 0; w < 3; w++) fn();
        CK(hipDeviceSynchronize());
        const int R = 20; float ms = 0;
        CK(hipEventRecord(a)); for (int r = 0; r < R; r++) fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b)); ms /= R;
        printf("%-44s %9.1f us  %8.1f GB/s(useful)  %7.2f G ops/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9, (double)M / (ms * 1e-3) / 1e9);
        return 0;
    };
    dim3 g(8192), blk(256);
    T("empty kernel", 0, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0); });
    T("empty kernel 9766 x 256", 0, [&] { hipLaunchKernelGGL(empty_kernel, dim3(9766), dim3(256), 0, 0); });
    T("empty kernel 9766 x 256, 20 KB LDS", 0, [&] { hipLaunchKernelGGL(empty_kernel, dim3(9766), dim3(256), 20480, 0); });
    T("idle chunks 9766 (flags load, 20 KB LDS)", 0, [&] { hipLaunchKernelGGL(idle_chunks, dim3(9766), dim3(256), 20480, 0, flags, cnt); });
    T("idle chunks 9766, 3-load chain", 0, [&] { hipLaunchKernelGGL(idle_chain, dim3(9766), dim3(256), 20480, 0, flags, buf, cnt); });
    T("idle chunks 2442 x 4096 vertices", 0, [&] { hipLaunchKernelGGL(idle_chunks, dim3(2442), dim3(256), 20480, 0, flags, cnt); });
    T("copy 128-bit 200MB->200MB", 2.0 * E * 4, [&] { hipLaunchKernelGGL(copy128, g, blk, 0, 0, (uint4*)out, (const uint4*)buf, E / 4); });
    T("scatter 4B into 200MB (26M)", 4.0 * M, [&] { hipLaunchKernelGGL(scatter32, g, blk, 0, 0, buf, idx, M); });
    T("gather 4B from 200MB (26M)", 4.0 * M, [&] { hipLaunchKernelGGL(gather32, g, blk, 0, 0, out, buf, idx, M); });
    T("scatter 1B into 10MB  (26M)", 1.0 * M, [&] { hipLaunchKernelGGL(scatter8, g, blk, 0, 0, flags, idx, M, (1u << 23) - 1); });
    T("scatter 1B into 1MB   (26M)", 1.0 * M, [&] { hipLaunchKernelGGL(scatter8, g, blk, 0, 0, flags, idx, M, (1u << 20) - 1); });
    T("scatter 1B into 128KB (26M)", 1.0 * M, [&] { hipLaunchKernelGGL(scatter8, g, blk, 0, 0, flags, idx, M, (1u << 17) - 1); });
    T("scan 1B/thread 10MB", 1.0 * N, [&] { hipLaunchKernelGGL(scan8, g, blk, 0, 0, flags, N, cnt); });
    T("scan 16B/thread 10MB", 1.0 * N, [&] { hipLaunchKernelGGL(scan128, dim3(2048), blk, 0, 0, (const uint4*)flags, N / 16, cnt); });
    T("scan 16B/thread 200MB", 4.0 * E, [&] { hipLaunchKernelGGL(scan128, g, blk, 0, 0, (const uint4*)buf, E / 4, cnt); });
    // working-set sizes for a narrower inbox (u8 / u16 words) and sender-state gathers
    uint8_t* b8; CK(hipMalloc(&b8, E));
    T("scatter 1B into 50MB  (26M)", 1.0 * M, [&] { hipLaunchKernelGGL(scatter8m, g, blk, 0, 0, b8, idx, M, E); });
    T("scatter 2B into 100MB (26M)", 2.0 * M, [&] { hipLaunchKernelGGL(scatter16, g, blk, 0, 0, (uint16_t*)buf, idx, M, E); });
    T("scatter 4B into 50MB  (26M)", 4.0 * M, [&] { hipLaunchKernelGGL(scatter16, g, blk, 0, 0, (uint16_t*)buf, idx, M, E / 2); });
    T("gather 16B from 160MB (26M)", 16.0 * M, [&] { hipLaunchKernelGGL(gather128, g, blk, 0, 0, (uint4*)out, (const uint4*)buf, idx, M, N); });
    // region-grouped: targets grouped by 256 KB region, random inside it
    {
        std::vector<uint32_t> hr(h);
        std::stable_sort(hr.begin(), hr.end(), [](uint32_t x, uint32_t y) { return (x >> 16) < (y >> 16); });
        std::vector<uint32_t> tmp(hr);
        // shuffle inside each region so the writes are not sequential
        for (size_t i = 0; i < hr.size();) {
            size_t j = i;
            while (j < hr.size() && (hr[j] >> 16) == (hr[i] >> 16)) j++;
            std::shuffle(hr.begin() + i, hr.begin() + j, rng);
            i = j;
        }
        CK(hipMemcpy(idx, hr.data(), M * 4, hipMemcpyHostToDevice));
        T("scatter 4B into 200MB, 256KB-region grouped", 4.0 * M, [&] { hipLaunchKernelGGL(scatter32, g, blk, 0, 0, buf, idx, M); });
        CK(hipMemcpy(idx, h.data(), M * 4, hipMemcpyHostToDevice));
    }
    // sorted-within-chunk scatter: idx sorted in 64K windows (locality)
    std::vector<uint32_t> hs(h);
    for (uint32_t i = 0; i < M; i += 65536) std::sort(hs.begin() + i, hs.begin() + std::min<uint32_t>(M, i + 65536));
    CK(hipMemcpy(idx, hs.data(), M * 4, hipMemcpyHostToDevice));
    T("scatter 4B into 200MB, 64K-window sorted", 4.0 * M, [&] { hipLaunchKernelGGL(scatter32, g, blk, 0, 0, buf, idx, M); });
    std::sort(hs.begin(), hs.end());
    CK(hipMemcpy(idx, hs.data(), M * 4, hipMemcpyHostToDevice));
    T("scatter 4B into 200MB, fully sorted", 4.0 * M, [&] { hipLaunchKernelGGL(scatter32, g, blk, 0, 0, buf, idx, M); });
    return 0;
}
