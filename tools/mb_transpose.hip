// Micro-benchmark (round 4): the dense-round message transport of the 10M
// Plumtree flood as a two-pass, XCD-local transpose instead of one random
// 4-byte store per message.
//
// Shape: E = 50M slots (10M vertices x 5), a fixed permutation tgt[] from
// sender slot to receiver slot (the overlay's reverse slots), a fraction of
// the sender slots carrying a word this round (r12 of the flood: 54 %).
//   direct : inbox[tgt[e]] = word[e] for the slots with a word (today's path)
//   pass 1 : per 5120-slot sender chunk (one 256-thread workgroup), the words
//            are permuted in LDS into bucket order (B receiver buckets, each
//            a contiguous range of receiver slots) and written out as one run
//            per (bucket, chunk) segment:
//              D: dense, every slot's word (0 = none) at a static position,
//                 pass 2 reads a static receiver slot per position
//              R: compacted 8-byte records {receiver slot, word} + a count
//                 per segment
//   pass 2 : workgroups read their XCD id (HW_REG_XCC_ID) and take (bucket,
//            part) work items of that XCD's buckets from a per-XCD counter,
//            in bucket order, so an XCD's stores land in one L2-sized window
//            of the inbox at a time.
// hipcc --offload-arch=gfx950 -O3 -o /tmp/mbt tools/mb_transpose.hip && /tmp/mbt
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr uint32_t kChunk = 5120;      // sender slots per workgroup (1024 vertices x 5)
constexpr uint32_t kMaxB = 512;

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}

__global__ __launch_bounds__(256) void k_exit(const uint32_t* __restrict__ flag, uint32_t* sink) {
    __shared__ uint32_t f;
    if (threadIdx.x == 0) f = flag[0];
    __syncthreads();
    if (f == 0) return;
    sink[blockIdx.x] = f;
}

__global__ __launch_bounds__(256) void k_read(const uint32_t* __restrict__ word, const uint32_t* __restrict__ tgt,
                                              uint32_t E, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < E; e += gridDim.x * 256) acc += word[e] ^ tgt[e];
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_direct(const uint32_t* __restrict__ word, const uint32_t* __restrict__ tgt,
                                                uint32_t E, uint32_t* __restrict__ inbox) {
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < E; e += gridDim.x * 256) {
        const uint32_t w = word[e];
        if (w) inbox[tgt[e]] = w;
    }
}

// destination-range split: one pass of P writes only the
// words whose receiver slot lies in [lo, lo + span)
__global__ __launch_bounds__(256) void k_range(const uint32_t* __restrict__ word, const uint32_t* __restrict__ tgt,
                                               uint32_t E, uint32_t lo, uint32_t span, uint32_t* __restrict__ inbox) {
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < E; e += gridDim.x * 256) {
        const uint32_t w = word[e], t = tgt[e];
        if (w && t - lo < span) inbox[t] = w;
    }
}

// pass 1, dense: image position of slot e = segbase[c][b(e)] + rank8[e]
__global__ __launch_bounds__(256) void k_p1_dense(const uint32_t* __restrict__ word, const uint32_t* __restrict__ tgt,
                                                  const uint8_t* __restrict__ rank8, const uint16_t* __restrict__ segbase,
                                                  const uint32_t* __restrict__ off, uint32_t E, uint32_t B,
                                                  uint32_t bshift, uint32_t C, uint32_t* __restrict__ X) {
    __shared__ uint32_t img[kChunk];
    __shared__ uint16_t sb[kMaxB + 1];
    __shared__ uint8_t bof[kChunk];
    const uint32_t c = blockIdx.x, t = threadIdx.x;
    const uint32_t e0 = c * kChunk, ne = min(kChunk, E - e0);
    for (uint32_t b = t; b <= B; b += 256) sb[b] = segbase[size_t(c) * (B + 1) + b];
    __syncthreads();
    for (uint32_t i = t; i < ne; i += 256) {
        const uint32_t e = e0 + i;
        const uint32_t b = tgt[e] >> bshift;
        const uint32_t p = sb[b] + rank8[e];
        img[p] = word[e];
        bof[p] = (uint8_t)b;
    }
    __syncthreads();
    for (uint32_t i = t; i < ne; i += 256) {
        const uint32_t b = bof[i];
        X[off[size_t(b) * C + c] + (i - sb[b])] = img[i];
    }
}

// pass 2, dense: work item = (bucket, range of X positions); a per-XCD queue
__global__ __launch_bounds__(256) void k_p2_dense(const uint32_t* __restrict__ X, const uint32_t* __restrict__ tgt2,
                                                  const uint64_t* __restrict__ boff, uint32_t B, uint32_t parts,
                                                  uint32_t* __restrict__ qhead, uint32_t* __restrict__ inbox) {
    __shared__ uint32_t item;
    const uint32_t x = xcc_id(), t = threadIdx.x;
    const uint32_t nb = (B + 7 - x) / 8;                 // buckets x, x+8, ...
    for (;;) {
        if (t == 0) item = atomicAdd(&qhead[x * 32], 1u);
        __syncthreads();
        const uint32_t it = item;
        __syncthreads();
        if (it >= nb * parts) break;
        const uint32_t b = x + 8 * (it / parts), p = it % parts;
        const uint64_t lo = boff[b], hi = boff[b + 1], len = hi - lo;
        const uint64_t a = lo + len * p / parts, z = lo + len * (p + 1) / parts;
        for (uint64_t i = a + t; i < z; i += 256) {
            const uint32_t w = __builtin_nontemporal_load(&X[i]);
            if (w) inbox[__builtin_nontemporal_load(&tgt2[i])] = w;
        }
    }
}

// pass 1, records: only the slots with a word; position in its segment by an
// LDS counter per bucket (order inside a segment is irrelevant: the record
// carries its receiver slot); cnt[b][c] = records written
__global__ __launch_bounds__(256) void k_p1_rec(const uint32_t* __restrict__ word, const uint32_t* __restrict__ tgt,
                                                const uint16_t* __restrict__ segbase, const uint32_t* __restrict__ off,
                                                uint32_t E, uint32_t B, uint32_t bshift, uint32_t C,
                                                uint2* __restrict__ X8, uint16_t* __restrict__ cnt) {
    __shared__ uint2 img[kChunk];
    __shared__ uint16_t sb[kMaxB + 1];
    __shared__ uint32_t fill[kMaxB];
    __shared__ uint32_t nimg;
    __shared__ uint32_t lst[kChunk];            // image index -> b, position
    const uint32_t c = blockIdx.x, t = threadIdx.x;
    const uint32_t e0 = c * kChunk, ne = min(kChunk, E - e0);
    for (uint32_t b = t; b <= B; b += 256) sb[b] = segbase[size_t(c) * (B + 1) + b];
    for (uint32_t b = t; b < B; b += 256) fill[b] = 0;
    for (uint32_t i = t; i < kChunk; i += 256) lst[i] = 0;
    if (t == 0) nimg = 0;
    __syncthreads();
    for (uint32_t i = t; i < ne; i += 256) {
        const uint32_t e = e0 + i;
        const uint32_t w = word[e];
        if (!w) continue;
        const uint32_t r = tgt[e], b = r >> bshift;
        const uint32_t k = atomicAdd(&fill[b], 1u);
        img[sb[b] + k] = make_uint2(r, w);
    }
    __syncthreads();
    for (uint32_t b = t; b < B; b += 256) cnt[size_t(b) * C + c] = (uint16_t)fill[b];
    // copy-out: image index i belongs to bucket b with sb[b] <= i < sb[b] + fill[b]
    for (uint32_t b = t; b < B; b += 256) {
        const uint32_t f = fill[b];
        for (uint32_t k = 0; k < f; k++) lst[sb[b] + k] = b | 0x80000000u;
    }
    __syncthreads();
    for (uint32_t i = t; i < ne; i += 256) {
        const uint32_t l = lst[i];
        if (!(l >> 31)) continue;
        const uint32_t b = l & 0xFFFFu;
        if (b >= B || i - sb[b] >= fill[b]) continue;
        X8[off[size_t(b) * C + c] + (i - sb[b])] = img[i];
    }
    (void)nimg;
}

__global__ __launch_bounds__(256) void k_p2_rec(const uint2* __restrict__ X8, const uint16_t* __restrict__ cnt,
                                                const uint32_t* __restrict__ off, uint32_t B, uint32_t C,
                                                uint32_t cper, uint32_t* __restrict__ qhead,
                                                uint32_t* __restrict__ inbox) {
    __shared__ uint32_t item;
    __shared__ uint32_t pre[257];
    const uint32_t x = xcc_id(), t = threadIdx.x;
    const uint32_t nb = (B + 7 - x) / 8, parts = (C + cper - 1) / cper;
    for (;;) {
        if (t == 0) item = atomicAdd(&qhead[x * 32], 1u);
        __syncthreads();
        const uint32_t it = item;
        if (it >= nb * parts) break;
        const uint32_t b = x + 8 * (it / parts), c0 = (it % parts) * cper, c1 = min(C, c0 + cper);
        if (t == 0) {
            uint32_t acc = 0;
            for (uint32_t c = c0; c < c1; c++) { pre[c - c0] = acc; acc += cnt[size_t(b) * C + c]; }
            pre[c1 - c0] = acc;
        }
        __syncthreads();
        const uint32_t tot = pre[c1 - c0];
        for (uint32_t i = t; i < tot; i += 256) {
            uint32_t lo = 0, hi = c1 - c0;
            while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (pre[m] <= i) lo = m; else hi = m; }
            const uint2 r = X8[off[size_t(b) * C + c0 + lo] + (i - pre[lo])];
            inbox[r.x] = r.y;
        }
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    const uint32_t N = 10'000'000, W = 5, E = N * W;
    const double frac = argc > 1 ? atof(argv[1]) : 0.54;
    const uint32_t C = (E + kChunk - 1) / kChunk;
    std::mt19937_64 rng(7);
    std::vector<uint32_t> tgt(E), word(E);
    std::iota(tgt.begin(), tgt.end(), 0u);
    std::shuffle(tgt.begin(), tgt.end(), rng);
    std::bernoulli_distribution on(frac);
    uint64_t M = 0;
    for (uint32_t e = 0; e < E; e++) { word[e] = on(rng) ? (e | 1u) : 0u; M += word[e] != 0; }
    printf("E=%u slots, %llu words (%.0f %%), %u chunks\n", E, (unsigned long long)M, 100.0 * M / E, C);
    uint32_t *d_tgt, *d_word, *d_inbox, *d_X, *d_tgt2, *d_off, *d_q, *d_sink;
    uint8_t* d_rank8;
    uint16_t *d_segbase, *d_cnt;
    uint64_t* d_boff;
    uint2* d_X8;
    CK(hipMalloc(&d_tgt, E * 4ull)); CK(hipMalloc(&d_word, E * 4ull)); CK(hipMalloc(&d_inbox, E * 4ull));
    CK(hipMalloc(&d_X, E * 4ull)); CK(hipMalloc(&d_tgt2, E * 4ull)); CK(hipMalloc(&d_rank8, E));
    CK(hipMalloc(&d_X8, E * 8ull)); CK(hipMalloc(&d_q, 8 * 32 * 4)); CK(hipMalloc(&d_sink, 4));
    CK(hipMemcpy(d_tgt, tgt.data(), E * 4ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_word, word.data(), E * 4ull, hipMemcpyHostToDevice));
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
    {
        uint32_t* d_flag;
        CK(hipMalloc(&d_flag, 4));
        CK(hipMemset(d_flag, 0, 4));
        for (uint32_t g : {256u, 1536u, 9766u}) {
            const float te = timeit([&] {
                for (int k = 0; k < 16; k++) hipLaunchKernelGGL(k_exit, dim3(g), dim3(256), 0, 0, d_flag, d_inbox);
            });
            printf("early-exit kernel, grid %5u: %5.2f us per launch (16 back to back)\n", g, te / 16);
        }
    }
    const float tr = timeit([&] { hipLaunchKernelGGL(k_read, dim3(cus * 8), dim3(256), 0, 0, d_word, d_tgt, E, d_sink); });
    const float td = timeit([&] { hipLaunchKernelGGL(k_direct, dim3(cus * 8), dim3(256), 0, 0, d_word, d_tgt, E, d_inbox); });
    printf("read word+tgt (400 MB)        %7.1f us\n", tr);
    printf("direct scatter                %7.1f us  (%.1f G words/s)\n", td, M / td / 1e3);
    std::vector<uint32_t> ref(E, 0);
    for (uint32_t e = 0; e < E; e++) if (word[e]) ref[tgt[e]] = word[e];
    for (uint32_t P : {2u, 4u, 8u}) {
        const uint32_t span = (E + P - 1) / P;
        CK(hipMemset(d_inbox, 0, E * 4ull));
        const float tp = timeit([&] {
            for (uint32_t p = 0; p < P; p++)
                hipLaunchKernelGGL(k_range, dim3(cus * 8), dim3(256), 0, 0, d_word, d_tgt, E, p * span, span, d_inbox);
        });
        std::vector<uint32_t> got(E);
        CK(hipMemcpy(got.data(), d_inbox, E * 4ull, hipMemcpyDeviceToHost));
        printf("range split P=%u (%.0f MB windows)  %7.1f us  (%.1f G words/s)  %s\n", P, span * 4.0 / 1e6, tp,
               M / tp / 1e3, got == ref ? "ok" : "MISMATCH");
    }
    for (uint32_t bshift : {22u, 21u, 20u, 19u}) {
        const uint32_t B = (E + (1u << bshift) - 1) >> bshift;
        if (B > kMaxB || B > 256) continue;      // bof is u8
        // static layout: segments (b, c) in b-major order; rank of a slot in its segment (sender order)
        std::vector<uint32_t> cntbc(size_t(B) * C, 0);
        std::vector<uint8_t> rank8(E);
        std::vector<uint16_t> segbase(size_t(C) * (B + 1));
        uint32_t maxseg = 0;
        for (uint32_t c = 0; c < C; c++) {
            const uint32_t e0 = c * kChunk, ne = std::min(kChunk, E - e0);
            std::vector<uint32_t> k(B, 0);
            for (uint32_t i = 0; i < ne; i++) {
                const uint32_t b = tgt[e0 + i] >> bshift;
                rank8[e0 + i] = (uint8_t)k[b]++;
            }
            uint32_t acc = 0;
            for (uint32_t b = 0; b < B; b++) {
                segbase[size_t(c) * (B + 1) + b] = (uint16_t)acc;
                acc += k[b];
                cntbc[size_t(b) * C + c] = k[b];
                maxseg = std::max(maxseg, k[b]);
            }
            segbase[size_t(c) * (B + 1) + B] = (uint16_t)acc;
        }
        if (maxseg > 255) { printf("B=%u: a segment of %u slots (rank8 overflows), skipped\n", B, maxseg); continue; }
        std::vector<uint32_t> off(size_t(B) * C);
        std::vector<uint64_t> boff(B + 1);
        uint64_t acc = 0;
        for (uint32_t b = 0; b < B; b++) {
            boff[b] = acc;
            for (uint32_t c = 0; c < C; c++) { off[size_t(b) * C + c] = (uint32_t)acc; acc += cntbc[size_t(b) * C + c]; }
        }
        boff[B] = acc;
        std::vector<uint32_t> tgt2(E);
        for (uint32_t c = 0; c < C; c++) {
            const uint32_t e0 = c * kChunk, ne = std::min(kChunk, E - e0);
            for (uint32_t i = 0; i < ne; i++) {
                const uint32_t b = tgt[e0 + i] >> bshift;
                tgt2[off[size_t(b) * C + c] + rank8[e0 + i]] = tgt[e0 + i];
            }
        }
        CK(hipMalloc(&d_segbase, segbase.size() * 2)); CK(hipMalloc(&d_off, off.size() * 4));
        CK(hipMalloc(&d_boff, boff.size() * 8)); CK(hipMalloc(&d_cnt, size_t(B) * C * 2));
        CK(hipMemcpy(d_segbase, segbase.data(), segbase.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_boff, boff.data(), boff.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_rank8, rank8.data(), E, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_tgt2, tgt2.data(), E * 4ull, hipMemcpyHostToDevice));
        const float t1 = timeit([&] {
            hipLaunchKernelGGL(k_p1_dense, dim3(C), dim3(256), 0, 0, d_word, d_tgt, d_rank8, d_segbase, d_off, E, B,
                               bshift, C, d_X);
        });
        for (uint32_t parts : {8u, 32u}) {
            for (uint32_t wpc : {4u, 8u}) {
                CK(hipMemset(d_inbox, 0, E * 4ull));
                const float t2 = timeit([&] {
                    (void)hipMemsetAsync(d_q, 0, 8 * 32 * 4, 0);
                    hipLaunchKernelGGL(k_p2_dense, dim3(cus * wpc), dim3(256), 0, 0, d_X, d_tgt2, d_boff, B, parts,
                                       d_q, d_inbox);
                });
                std::vector<uint32_t> got(E);
                CK(hipMemcpy(got.data(), d_inbox, E * 4ull, hipMemcpyDeviceToHost));
                const bool ok = got == ref;
                printf("D B=%3u (%.2f MB windows) p1 %6.1f  p2(parts %2u, %u WG/CU) %6.1f  total %6.1f us  %s\n", B,
                       4.0 * (1u << bshift) / 1e6, t1, parts, wpc, t2, t1 + t2, ok ? "ok" : "MISMATCH");
            }
        }
        const float t1r = timeit([&] {
            hipLaunchKernelGGL(k_p1_rec, dim3(C), dim3(256), 0, 0, d_word, d_tgt, d_segbase, d_off, E, B, bshift, C,
                               d_X8, d_cnt);
        });
        for (uint32_t cper : {64u, 256u}) {
            CK(hipMemset(d_inbox, 0, E * 4ull));
            const float t2r = timeit([&] {
                (void)hipMemsetAsync(d_q, 0, 8 * 32 * 4, 0);
                hipLaunchKernelGGL(k_p2_rec, dim3(cus * 4), dim3(256), 0, 0, d_X8, d_cnt, d_off, B, C, cper, d_q,
                                   d_inbox);
            });
            std::vector<uint32_t> got(E);
            CK(hipMemcpy(got.data(), d_inbox, E * 4ull, hipMemcpyDeviceToHost));
            const bool ok = got == ref;
            printf("R B=%3u p1 %6.1f  p2(%3u chunks per item) %6.1f  total %6.1f us  %s\n", B, t1r, cper, t2r,
                   t1r + t2r, ok ? "ok" : "MISMATCH");
        }
        CK(hipFree(d_segbase)); CK(hipFree(d_off)); CK(hipFree(d_boff)); CK(hipFree(d_cnt));
    }
    return 0;
}
