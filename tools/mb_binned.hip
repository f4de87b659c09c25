// Micro-benchmark (round 4): the dense-round message transport as three
// coalesced passes with every random access inside LDS, against today's one
// random 4-byte store per message.  Shape: r12 of the 10M-peer flood --
// E = 50M receiver slots, a fixed permutation tgt[] (sender slot -> receiver
// slot), 54 % of the sender slots carrying a word.
//   P1 sender chunk (5120 slots) -> 64 coarse buckets: LDS rank per bucket,
//      8-byte records {receiver slot, word} written as one run per (bucket,
//      chunk) segment (static capacity = the chunk's slots into that bucket)
//   P2 (coarse bucket, 32 chunks) -> 64 fine windows of that bucket: the same
//   P3 fine window (12,208 slots, 48.8 KB): records scattered into an LDS
//      image of the window, written out whole (in the round kernel the
//      window's vertices would be handled from LDS instead)
// hipcc --offload-arch=gfx950 -O3 -o tools/mb_binned tools/mb_binned.hip && tools/mb_binned
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr uint32_t kChunk = 5120;   // sender slots per P1 workgroup
constexpr uint32_t kB = 64;         // coarse buckets
constexpr uint32_t kF = 64;         // fine windows per coarse bucket
constexpr uint32_t kCpi = 32;       // sender chunks per P2 item
constexpr uint32_t kImg = 6144;     // P2 LDS records (>= max records of an item)

__global__ __launch_bounds__(256) void k_direct(const uint32_t* __restrict__ word, const uint32_t* __restrict__ tgt,
                                                uint32_t E, uint32_t* __restrict__ inbox) {
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < E; e += gridDim.x * 256) {
        const uint32_t w = word[e];
        if (w) inbox[tgt[e]] = w;
    }
}

// P1: grid = chunks
__global__ __launch_bounds__(256) void k_p1(const uint32_t* __restrict__ word, const uint32_t* __restrict__ tgt,
                                            uint32_t E, uint32_t cslots, const uint16_t* __restrict__ sb1,
                                            const uint32_t* __restrict__ off1, uint32_t C, uint2* __restrict__ X1,
                                            uint16_t* __restrict__ cnt1) {
    __shared__ uint2 img[kChunk];
    __shared__ uint8_t bof[kChunk];
    __shared__ uint32_t fill[kB];
    __shared__ uint16_t sb[kB + 1];
    const uint32_t c = blockIdx.x, t = threadIdx.x;
    const uint32_t e0 = c * kChunk, ne = min(kChunk, E - e0);
    if (t < kB) fill[t] = 0;
    if (t <= kB) sb[t] = sb1[size_t(c) * (kB + 1) + t];
    for (uint32_t i = t; i < kChunk; i += 256) bof[i] = 0xFF;
    __syncthreads();
    constexpr uint32_t kPer = kChunk / 256;        // 20 slots per thread, all loads in flight at once
    uint32_t w[kPer], r[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        const uint32_t i = t + 256 * k;
        w[k] = i < ne ? word[e0 + i] : 0u;
        r[k] = i < ne ? tgt[e0 + i] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        if (!w[k]) continue;
        const uint32_t b = r[k] / cslots;
        const uint32_t p = sb[b] + atomicAdd(&fill[b], 1u);
        img[p] = make_uint2(r[k], w[k]);
        bof[p] = (uint8_t)b;
    }
    __syncthreads();
    if (t < kB) cnt1[size_t(t) * C + c] = (uint16_t)fill[t];
    for (uint32_t i = t; i < ne; i += 256) {
        const uint32_t b = bof[i];
        if (b == 0xFF) continue;
        X1[off1[size_t(b) * C + c] + (i - sb[b])] = img[i];
    }
}

// P2: grid = kB * items; item = chunks [it * kCpi, ...) of bucket b
__global__ __launch_bounds__(256) void k_p2(const uint2* __restrict__ X1, const uint16_t* __restrict__ cnt1,
                                            const uint32_t* __restrict__ off1, uint32_t C, uint32_t items,
                                            uint32_t cslots, uint32_t fslots, const uint16_t* __restrict__ sb2,
                                            const uint32_t* __restrict__ off2, uint2* __restrict__ X2,
                                            uint16_t* __restrict__ cnt2) {
    __shared__ uint2 img[kImg];
    __shared__ uint8_t bof[kImg];
    __shared__ uint32_t fill[kF];
    __shared__ uint16_t sb[kF + 1];
    __shared__ uint32_t pre[kCpi + 1], src[kCpi];
    const uint32_t b = blockIdx.x / items, it = blockIdx.x % items, t = threadIdx.x;
    const uint32_t c0 = it * kCpi, nc = min(kCpi, C - c0);
    if (t < kF) fill[t] = 0;
    if (t <= kF) sb[t] = sb2[(size_t(b) * items + it) * (kF + 1) + t];
    for (uint32_t i = t; i < kImg; i += 256) bof[i] = 0xFF;
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t k = 0; k < nc; k++) {
            pre[k] = acc;
            src[k] = off1[size_t(b) * C + c0 + k];
            acc += cnt1[size_t(b) * C + c0 + k];
        }
        pre[nc] = acc;
    }
    __syncthreads();
    const uint32_t tot = pre[nc], rbase = b * cslots;
    constexpr uint32_t kPer = kImg / 256;          // 24 records per thread, all loads in flight at once
    uint2 rr[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        const uint32_t i = t + 256 * k;
        uint32_t lo = 0, hi = nc;
        while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (pre[m] <= i) lo = m; else hi = m; }
        rr[k] = i < tot ? X1[src[lo] + (i - pre[lo])] : make_uint2(0xFFFFFFFFu, 0u);
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        if (rr[k].x == 0xFFFFFFFFu) continue;
        const uint32_t f = (rr[k].x - rbase) / fslots;
        const uint32_t p = sb[f] + atomicAdd(&fill[f], 1u);
        img[p] = rr[k];
        bof[p] = (uint8_t)f;
    }
    __syncthreads();
    if (t < kF) cnt2[(size_t(b) * kF + t) * items + it] = (uint16_t)fill[t];
    const uint32_t cap = sb[kF];
    for (uint32_t i = t; i < cap; i += 256) {
        const uint32_t f = bof[i];
        if (f == 0xFF) continue;
        X2[off2[(size_t(b) * kF + f) * items + it] + (i - sb[f])] = img[i];
    }
}

// P3: grid = kB * kF windows
__global__ __launch_bounds__(256) void k_p3(const uint2* __restrict__ X2, const uint16_t* __restrict__ cnt2,
                                            const uint32_t* __restrict__ off2, uint32_t items, uint32_t cslots,
                                            uint32_t fslots, uint32_t E, uint32_t* __restrict__ inbox) {
    extern __shared__ uint32_t win[];
    __shared__ uint32_t pre[1024 + 1], src[1024];
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    const uint32_t b = g / kF, f = g % kF;
    const uint32_t lo_slot = b * cslots + f * fslots;
    const uint32_t ns = min(fslots, min(E, (b + 1) * cslots) - min(lo_slot, min(E, (b + 1) * cslots)));
    for (uint32_t i = t; i < fslots; i += 256) win[i] = 0;
    for (uint32_t k = t; k < items; k += 256) {
        src[k] = off2[size_t(g) * items + k];
        pre[k + 1] = cnt2[size_t(g) * items + k];
    }
    if (t == 0) pre[0] = 0;
    __syncthreads();
    if (t == 0)
        for (uint32_t k = 1; k <= items; k++) pre[k] += pre[k - 1];
    __syncthreads();
    const uint32_t tot = pre[items];
    constexpr uint32_t kPer = 16;                  // records per thread per batch, loads in flight at once
    for (uint32_t base = 0; base < tot; base += 256 * kPer) {
        uint2 rr[kPer];
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t i = base + t + 256 * k;
            uint32_t lo = 0, hi = items;
            while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (pre[m] <= i) lo = m; else hi = m; }
            rr[k] = i < tot ? X2[src[lo] + (i - pre[lo])] : make_uint2(0xFFFFFFFFu, 0u);
        }
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++)
            if (rr[k].x != 0xFFFFFFFFu) win[rr[k].x - lo_slot] = rr[k].y;
    }
    __syncthreads();
    for (uint32_t i = t; i < ns; i += 256) inbox[lo_slot + i] = win[i];
}

int main() {
    const uint32_t N = 10'000'000, W = 5, E = N * W;
    const uint32_t C = (E + kChunk - 1) / kChunk;
    const uint32_t cslots = (E + kB - 1) / kB, fslots = (cslots + kF - 1) / kF;
    const uint32_t items = (C + kCpi - 1) / kCpi;
    std::mt19937_64 rng(7);
    std::vector<uint32_t> tgt(E), word(E);
    std::iota(tgt.begin(), tgt.end(), 0u);
    std::shuffle(tgt.begin(), tgt.end(), rng);
    std::bernoulli_distribution on(0.54);
    uint64_t M = 0;
    for (uint32_t e = 0; e < E; e++) { word[e] = on(rng) ? (e | 1u) : 0u; M += word[e] != 0; }
    printf("E=%u, %llu words, C=%u chunks, coarse %u slots, fine %u slots (%.1f KB), %u P2 items per bucket\n", E,
           (unsigned long long)M, C, cslots, fslots, fslots * 4 / 1024.0, items);
    if (items > 1024) { printf("too many items\n"); return 1; }
    // static capacities: P1 segments (b, c), P2 segments (b, item, f)
    std::vector<uint32_t> cap1(size_t(kB) * C, 0), cap2(size_t(kB) * items * kF, 0);
    for (uint32_t e = 0; e < E; e++) {
        const uint32_t c = e / kChunk, b = tgt[e] / cslots, f = (tgt[e] - b * cslots) / fslots;
        cap1[size_t(b) * C + c]++;
        cap2[(size_t(b) * items + c / kCpi) * kF + f]++;
    }
    std::vector<uint16_t> sb1(size_t(C) * (kB + 1)), sb2(size_t(kB) * items * (kF + 1));
    uint32_t mx1 = 0, mx2 = 0;
    for (uint32_t c = 0; c < C; c++) {
        uint32_t a = 0;
        for (uint32_t b = 0; b < kB; b++) { sb1[size_t(c) * (kB + 1) + b] = (uint16_t)a; a += cap1[size_t(b) * C + c]; }
        sb1[size_t(c) * (kB + 1) + kB] = (uint16_t)a;
        mx1 = std::max(mx1, a);
    }
    for (uint32_t b = 0; b < kB; b++)
        for (uint32_t it = 0; it < items; it++) {
            uint32_t a = 0;
            const size_t k = size_t(b) * items + it;
            for (uint32_t f = 0; f < kF; f++) { sb2[k * (kF + 1) + f] = (uint16_t)a; a += cap2[k * kF + f]; }
            sb2[k * (kF + 1) + kF] = (uint16_t)a;
            mx2 = std::max(mx2, a);
        }
    if (mx1 > kChunk || mx2 > kImg) { printf("capacity: %u %u\n", mx1, mx2); return 1; }
    std::vector<uint32_t> off1(size_t(kB) * C), off2(size_t(kB) * kF * items);
    {
        uint64_t a = 0;
        for (uint32_t b = 0; b < kB; b++)
            for (uint32_t c = 0; c < C; c++) { off1[size_t(b) * C + c] = (uint32_t)a; a += cap1[size_t(b) * C + c]; }
        a = 0;
        for (uint32_t b = 0; b < kB; b++)
            for (uint32_t f = 0; f < kF; f++)
                for (uint32_t it = 0; it < items; it++) {
                    off2[(size_t(b) * kF + f) * items + it] = (uint32_t)a;
                    a += cap2[(size_t(b) * items + it) * kF + f];
                }
    }
    uint32_t *d_tgt, *d_word, *d_inbox, *d_off1, *d_off2;
    uint16_t *d_sb1, *d_sb2, *d_cnt1, *d_cnt2;
    uint2 *d_X1, *d_X2;
    CK(hipMalloc(&d_tgt, E * 4ull)); CK(hipMalloc(&d_word, E * 4ull)); CK(hipMalloc(&d_inbox, E * 4ull));
    CK(hipMalloc(&d_X1, E * 8ull)); CK(hipMalloc(&d_X2, E * 8ull));
    CK(hipMalloc(&d_off1, off1.size() * 4)); CK(hipMalloc(&d_off2, off2.size() * 4));
    CK(hipMalloc(&d_sb1, sb1.size() * 2)); CK(hipMalloc(&d_sb2, sb2.size() * 2));
    CK(hipMalloc(&d_cnt1, size_t(kB) * C * 2)); CK(hipMalloc(&d_cnt2, size_t(kB) * kF * items * 2));
    CK(hipMemcpy(d_tgt, tgt.data(), E * 4ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_word, word.data(), E * 4ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_off1, off1.data(), off1.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_off2, off2.data(), off2.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sb1, sb1.data(), sb1.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sb2, sb2.data(), sb2.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemset(d_inbox, 0, E * 4ull));
    hipEvent_t ev0, ev1;
    CK(hipEventCreate(&ev0)); CK(hipEventCreate(&ev1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto timeit = [&](auto fn) -> float {
        for (int w = 0; w < 2; w++) fn();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(ev0);
        for (int it = 0; it < 10; it++) fn();
        (void)hipEventRecord(ev1);
        (void)hipEventSynchronize(ev1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ev0, ev1);
        return ms * 100.f;
    };
    const float td = timeit([&] { hipLaunchKernelGGL(k_direct, dim3(cus * 8), dim3(256), 0, 0, d_word, d_tgt, E, d_inbox); });
    printf("direct scatter           %7.1f us  (%.1f G words/s)\n", td, M / td / 1e3);
    std::vector<uint32_t> ref(E, 0);
    for (uint32_t e = 0; e < E; e++) if (word[e]) ref[tgt[e]] = word[e];
    const float t1 = timeit([&] {
        hipLaunchKernelGGL(k_p1, dim3(C), dim3(256), 0, 0, d_word, d_tgt, E, cslots, d_sb1, d_off1, C, d_X1, d_cnt1);
    });
    const float t2 = timeit([&] {
        hipLaunchKernelGGL(k_p2, dim3(kB * items), dim3(256), 0, 0, d_X1, d_cnt1, d_off1, C, items, cslots, fslots, d_sb2,
                           d_off2, d_X2, d_cnt2);
    });
    CK(hipMemset(d_inbox, 0, E * 4ull));
    const float t3 = timeit([&] {
        hipLaunchKernelGGL(k_p3, dim3(kB * kF), dim3(256), fslots * 4, 0, d_X2, d_cnt2, d_off2, items, cslots, fslots, E,
                           d_inbox);
    });
    std::vector<uint32_t> got(E);
    CK(hipMemcpy(got.data(), d_inbox, E * 4ull, hipMemcpyDeviceToHost));
    printf("P1 %7.1f  P2 %7.1f  P3 %7.1f  total %7.1f us  (%.2fx direct)  %s\n", t1, t2, t3, t1 + t2 + t3,
           td / (t1 + t2 + t3), got == ref ? "ok" : "MISMATCH");
    return 0;
}
