// mb_latency.hip -- dependent-load latency of ONE workgroup vs the same
// chain with every CU busy (is a single-workgroup kernel latency-starved by
// power management?).  Diagnostic for the frontier kernel.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mb_latency.hip -o /tmp/mb_latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <random>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// lane 0 of each workgroup chases `hops` pointers starting at its own slot
__global__ void chase(const uint32_t* __restrict__ nxt, uint32_t hops, uint32_t* out, unsigned long long* ticks) {
    if (threadIdx.x != 0) return;
    uint32_t p = uint32_t(uint64_t(blockIdx.x) * 7919u % (uint64_t(1) << 28));
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t i = 0; i < hops; i++) p = __builtin_nontemporal_load(nxt + p);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x] = p;
    if (blockIdx.x == 0) ticks[0] = t1 - t0;
}

// every lane of a 1024-thread workgroup chases its own chain
__global__ __launch_bounds__(1024) void chase_wide(const uint32_t* __restrict__ nxt, uint32_t hops, uint32_t* out,
                                                   unsigned long long* ticks) {
    uint32_t p = uint32_t((uint64_t(blockIdx.x) * 1024u + threadIdx.x) * 104729ull % (uint64_t(1) << 28));   // < n
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t i = 0; i < hops; i++) p = __builtin_nontemporal_load(nxt + p);
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 1024u + threadIdx.x] = p;
    if (blockIdx.x == 0 && threadIdx.x == 0) ticks[0] = t1 - t0;
}

// a busy-spinning grid on the other CUs (streams a buffer) while workgroup 0 chases
__global__ void chase_with_load(const uint32_t* __restrict__ nxt, uint32_t hops, uint32_t* out, unsigned long long* ticks,
                                const uint4* __restrict__ big, size_t nbig, uint4* sink) {
    if (blockIdx.x == 0) {
        if (threadIdx.x != 0) return;
        uint32_t p = 12345u;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t i = 0; i < hops; i++) p = __builtin_nontemporal_load(nxt + p);
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        out[0] = p;
        ticks[0] = t1 - t0;
        return;
    }
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t i = (size_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x; i < nbig; i += (size_t)(gridDim.x - 1) * blockDim.x) {
        const uint4 v = big[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if (acc.x == 0xFFFFFFFFu) sink[0] = acc;
}

// one lane: `k` operations to random addresses (all issued, then waited for), repeated `reps` times
// op 0: store, 1: non-returning device atomicOr, 2: returning atomicOr, 3: load
__global__ void ops_latency(uint32_t* __restrict__ buf, size_t n, uint32_t k, uint32_t reps, int op,
                            unsigned long long* ticks, uint32_t* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t x = 88172645463325252ull;
    uint32_t acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t r = 0; r < reps; r++) {
        for (uint32_t i = 0; i < k; i++) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            const size_t a = (size_t)(x % n);
            if (op == 0) buf[a] = (uint32_t)(x % n);   // the buffer is also the chase table: keep every entry < n
            else if (op == 1) atomicOr(buf + a, 1u);
            else if (op == 2) acc += atomicOr(buf + a, 1u);
            else acc += __builtin_nontemporal_load(buf + a);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    ticks[0] = t1 - t0;
    out[0] = acc;
}

// batches of `k` random loads, varying how they are spread: mode 0: one lane, k
// instructions; 1: k lanes of one wave, one instruction; 2: k waves of one
// workgroup, one lane each; 3: one lane, k loads inside one 64 KB window
// (random window per batch); 4: one lane, k loads inside one 2 MB window
__global__ __launch_bounds__(1024) void spread_latency(const uint32_t* __restrict__ buf, size_t n, uint32_t k,
                                                       uint32_t reps, int mode, unsigned long long* ticks, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const bool active = mode == 1 ? (wv == 0 && lane < k) : mode == 2 ? (lane == 0 && wv < k) : threadIdx.x == 0;
    uint64_t x = 88172645463325252ull + threadIdx.x * 7919ull;
    uint32_t acc = 0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t r = 0; r < reps; r++) {
        if (active) {
            if (mode == 0 || mode >= 3) {
                x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                const size_t win = (mode == 3 || mode == 6) ? 16384 : mode == 4 ? 524288 : n;
                const size_t base = (mode == 3 || mode == 4 || mode == 6) ? (size_t)(x % (n / win)) * win : 0;
                for (uint32_t i = 0; i < k; i++) {
                    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                    if (mode >= 5) acc += buf[base + (size_t)(x % win)];            // plain (cached) loads
                    else acc += __builtin_nontemporal_load(buf + base + (size_t)(x % win));
                }
            } else {
                x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                acc += __builtin_nontemporal_load(buf + (size_t)(x % n));
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) ticks[0] = t1 - t0;
    out[threadIdx.x] = acc;
}

// one lane, 8 independent loads issued back to back (unrolled, addresses first), then one wait
template <bool kNt>
__global__ void unrolled8(const uint32_t* __restrict__ buf, size_t n, uint32_t reps, unsigned long long* ticks, uint32_t* out) {
    if (threadIdx.x != 0) return;
    uint64_t x = 88172645463325252ull;
    uint32_t acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t r = 0; r < reps; r++) {
        size_t ad[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            ad[i] = (size_t)(x % n);
        }
        uint32_t v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = kNt ? __builtin_nontemporal_load(buf + ad[i]) : buf[ad[i]];
#pragma unroll
        for (int i = 0; i < 8; i++) acc += v[i];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    ticks[0] = t1 - t0;
    out[0] = acc;
}

int main() {
    const size_t n = size_t(1) << 28;   // 1 GiB of u32: every hop misses every cache
    std::vector<uint32_t> h(n);
    std::mt19937_64 g(1);
    for (size_t i = 0; i < n; i++) h[i] = uint32_t(g() % n);
    uint32_t *d, *out;
    unsigned long long* ticks;
    CHK(hipMalloc(&d, n * 4));
    CHK(hipMalloc(&out, 1u << 24));
    CHK(hipMalloc(&ticks, 64));
    CHK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    const size_t nbig = size_t(1) << 26;   // 1 GiB of uint4
    uint4 *big, *sink;
    CHK(hipMalloc(&big, nbig * 16));
    CHK(hipMemset(big, 1, nbig * 16));
    CHK(hipMalloc(&sink, 64));
    unsigned long long t;
    for (int op = 0; op < 4; op++)
        for (uint32_t k : {1u, 8u}) {
            const uint32_t reps = 200;
            hipLaunchKernelGGL(ops_latency, dim3(1), dim3(64), 0, 0, d, n, k, reps, op, ticks, out);
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
            static const char* nm[] = {"store", "atomicOr (no return)", "atomicOr (returned)", "nt load"};
            printf("%-22s x%u to random words of 1 GiB, then vmcnt(0): %.3f us per batch\n", nm[op], k,
                   t * 0.01 / reps);
        }
    for (int mode = 0; mode < 7; mode++) {
        const uint32_t reps = 200, k = 8;
        hipLaunchKernelGGL(spread_latency, dim3(1), dim3(1024), 0, 0, d, n, k, reps, mode, ticks, out);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
        static const char* nm[] = {"1 lane, 8 instructions", "8 lanes, 1 instruction", "8 waves x 1 lane",
                                   "1 lane, 8 in a 64 KB window", "1 lane, 8 in a 2 MB window",
                                   "1 lane, 8 plain loads", "1 lane, 8 plain in 64 KB"};
        printf("8 random loads, %-28s: %.3f us per batch\n", nm[mode], t * 0.01 / reps);
    }
    for (int nt = 0; nt < 2; nt++) {
        if (nt) hipLaunchKernelGGL(unrolled8<true>, dim3(1), dim3(64), 0, 0, d, n, 200u, ticks, out);
        else hipLaunchKernelGGL(unrolled8<false>, dim3(1), dim3(64), 0, 0, d, n, 200u, ticks, out);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
        printf("8 random loads, 1 lane, unrolled, all issued then one wait (%s): %.3f us per batch\n", nt ? "nt" : "plain",
               t * 0.01 / 200);
    }
    const uint32_t hops = 2000;
    for (int rep = 0; rep < 3; rep++) {
        for (uint32_t grid : {1u, 8u, 256u, 1024u}) {
            hipLaunchKernelGGL(chase, dim3(grid), dim3(64), 0, 0, d, hops, out, ticks);
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
            printf("chase: %4u workgroups x 1 lane: %.3f us per dependent load\n", grid, t * 0.01 / hops);
        }
        hipLaunchKernelGGL(chase_wide, dim3(1), dim3(1024), 0, 0, d, 200u, out, ticks);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
        printf("chase_wide: 1 workgroup x 1024 lanes: %.3f us per dependent step\n", t * 0.01 / 200);
        hipLaunchKernelGGL(chase_wide, dim3(256), dim3(1024), 0, 0, d, 200u, out, ticks);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
        printf("chase_wide: 256 workgroups x 1024 lanes: %.3f us per dependent step\n", t * 0.01 / 200);
        hipLaunchKernelGGL(chase_with_load, dim3(1024), dim3(256), 0, 0, d, hops, out, ticks, big, nbig, sink);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
        printf("chase beside a streaming grid: %.3f us per dependent load\n", t * 0.01 / hops);
    }
    return 0;
}
