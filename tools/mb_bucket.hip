// Micro-benchmark: can a dense round's random 4-byte word scatter (26.8M
// words into a 200 MB inbox, the r12 shape of a 10M-peer flood) be made
// cheaper by bucketing the words by receiver range first and applying each
// bucket from the L2 of one XCD?
//   direct : out[slot] = word, random (what the round kernel does)
//   phase 1: per 2744-word sender chunk (one 256-thread workgroup), an LDS
//            histogram over P receiver buckets, one reservation per bucket
//            in sub-region (b, chunk & 63), records {slot, word} written at
//            base + rank (runs of ~2744/P records)
//   phase 2: a resident grid; workgroups with equal blockIdx % 8 (one XCD)
//            walk the buckets b = label, label + 8, ... together, so an XCD
//            scatters into one 200 MB / P slice of the inbox at a time
// hipcc --offload-arch=gfx950 -O3 -o /tmp/mbb tools/mb_bucket.hip && /tmp/mbb
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr uint32_t kChunkMsgs = 2744;
constexpr uint32_t kSub = 64;

__global__ __launch_bounds__(256) void direct(uint32_t* __restrict__ out, const uint32_t* __restrict__ slot, uint32_t m) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < m; i += gridDim.x * 256) out[slot[i]] = i | 1u;
}

// one workgroup per chunk
__global__ __launch_bounds__(256) void phase1(const uint32_t* __restrict__ slot, uint32_t m, uint32_t shift, uint32_t P,
                                              const uint32_t* __restrict__ sub_base, uint32_t* __restrict__ cursor,
                                              uint2* __restrict__ rec) {
    __shared__ uint32_t hist[1024], base[1024];
    const uint32_t t = threadIdx.x, c = blockIdx.x;
    for (uint32_t b = t; b < P; b += 256) hist[b] = 0;
    __syncthreads();
    constexpr uint32_t kPer = (kChunkMsgs + 255) / 256;
    uint32_t s[kPer], r[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        const uint32_t i = c * kChunkMsgs + t + k * 256;
        s[k] = (t + k * 256 < kChunkMsgs && i < m) ? slot[i] : 0xFFFFFFFFu;
        r[k] = s[k] != 0xFFFFFFFFu ? atomicAdd(&hist[s[k] >> shift], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t b = t; b < P; b += 256)
        if (hist[b]) base[b] = sub_base[b * kSub + (c & (kSub - 1))] + atomicAdd(&cursor[b * kSub + (c & (kSub - 1))], hist[b]);
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++)
        if (s[k] != 0xFFFFFFFFu) rec[base[s[k] >> shift] + r[k]] = make_uint2(s[k], (c * kChunkMsgs + t + k * 256) | 1u);
}

// resident grid: group label x = blockIdx % 8, member j = blockIdx / 8 of G8
__global__ __launch_bounds__(256) void phase2(uint32_t* __restrict__ out, const uint2* __restrict__ rec,
                                              const uint32_t* __restrict__ sub_base, const uint32_t* __restrict__ cursor,
                                              uint32_t P) {
    __shared__ uint32_t pre[kSub + 1];
    const uint32_t x = blockIdx.x & 7, j = blockIdx.x >> 3, G8 = gridDim.x >> 3, t = threadIdx.x;
    for (uint32_t b = x; b < P; b += 8) {
        if (t == 0) {
            uint32_t acc = 0;
            for (uint32_t s = 0; s < kSub; s++) { pre[s] = acc; acc += cursor[b * kSub + s]; }
            pre[kSub] = acc;
        }
        __syncthreads();
        const uint32_t T = pre[kSub];
        for (uint32_t i = j * 256 + t; i < T; i += G8 * 256) {
            uint32_t lo = 0, hi = kSub;
            while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (pre[mid] <= i) lo = mid; else hi = mid; }
            const uint2 r = rec[sub_base[b * kSub + lo] + (i - pre[lo])];
            out[r.x] = r.y;
        }
        __syncthreads();
    }
}

int main() {
    const uint32_t E = 50'000'000, M = 26'800'000;
    const uint32_t nch = (M + kChunkMsgs - 1) / kChunkMsgs;
    std::vector<uint32_t> h(M);
    std::mt19937 rng(1);
    for (auto& x : h) x = rng() % E;
    uint32_t *slot, *out, *cursor, *sub_base;
    uint2* rec;
    CK(hipMalloc(&slot, M * 4ull)); CK(hipMalloc(&out, E * 4ull)); CK(hipMalloc(&rec, (M + 1024) * 8ull));
    CK(hipMalloc(&cursor, 1024 * kSub * 4)); CK(hipMalloc(&sub_base, 1024 * kSub * 4));
    CK(hipMemcpy(slot, h.data(), M * 4ull, hipMemcpyHostToDevice));
    CK(hipMemset(out, 0, E * 4ull));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto time = [&](auto fn) -> float {
        for (int w = 0; w < 2; w++) fn();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        for (int it = 0; it < 10; it++) fn();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        return ms * 100.f;   // us per call
    };
    const float td = time([&] { hipLaunchKernelGGL(direct, dim3(cus * 8), dim3(256), 0, 0, out, slot, M); });
    printf("direct random scatter 26.8M x 4B into 200 MB: %8.1f us  (%.1f G words/s)\n", td, M / td / 1e3);
    for (uint32_t shift : {21u, 20u, 19u, 18u}) {
        const uint32_t P = (E + (1u << shift) - 1) >> shift;
        if (P > 1024) continue;
        std::vector<uint32_t> cnt(size_t(P) * kSub, 0), base(size_t(P) * kSub, 0);
        for (uint32_t i = 0; i < M; i++) cnt[size_t(h[i] >> shift) * kSub + ((i / kChunkMsgs) & (kSub - 1))]++;
        uint32_t acc = 0;
        for (size_t k = 0; k < cnt.size(); k++) { base[k] = acc; acc += cnt[k]; }
        CK(hipMemcpy(sub_base, base.data(), base.size() * 4, hipMemcpyHostToDevice));
        const float t1 = time([&] {
            (void)hipMemsetAsync(cursor, 0, size_t(P) * kSub * 4, 0);
            hipLaunchKernelGGL(phase1, dim3(nch), dim3(256), 0, 0, slot, M, shift, P, sub_base, cursor, rec);
        });
        for (uint32_t per_cu : {4u, 8u}) {
            const float t2 = time([&] {
                hipLaunchKernelGGL(phase2, dim3(cus * per_cu), dim3(256), 0, 0, out, rec, sub_base, cursor, P);
            });
            printf("P=%4u buckets (%5.2f MB slices): phase1 %7.1f us  phase2(%u WG/CU) %7.1f us  total %7.1f us  (%.2fx direct)\n",
                   P, (4.0 * (1u << shift)) / 1e6, t1, per_cu, t2, t1 + t2, td / (t1 + t2));
        }
    }
    return 0;
}
