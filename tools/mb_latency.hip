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
            if (op == 0) buf[a] = (uint32_t)x;
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
