// mb_launch.hip -- what a sparse Plumtree round's floor is made of: the cost
// of one back-to-back launch of the resident round-kernel grid, against a
// device-wide barrier inside one persistent launch.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mb_launch.hip -o /tmp/mb_launch
//
// Every spin is bounded (a missed arrival sets err and the loop ends), so a
// grid that is not fully resident finishes with an error instead of hanging.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kBlock = 256;
constexpr uint32_t kSpinMax = 1u << 22;

// an empty workgroup with the round kernel's LDS footprint
__global__ __launch_bounds__(kBlock) void k_empty(uint32_t* out) {
    extern __shared__ uint32_t lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (lds[(threadIdx.x + 1) & (kBlock - 1)] == 0xFFFFFFFFu) out[0] = 1;
}

// what an idle workgroup of a sparse round does: read the 64 counts and the 64 list offsets, then leave
__global__ __launch_bounds__(kBlock) void k_counts(const uint32_t* __restrict__ cnt, uint32_t* out) {
    extern __shared__ uint32_t lds[];
    if (threadIdx.x < 128) lds[threadIdx.x] = cnt[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int i = 0; i < 128; i++) s += lds[i];
        if (s == 0xFFFFFFFFu) out[0] = s;
    }
}

// workgroup 0's lane 0 chases `hops` dependent pointers; the rest of the resident grid leaves
__global__ __launch_bounds__(kBlock) void k_chain(const uint32_t* __restrict__ nxt, uint32_t hops, uint32_t* out) {
    extern __shared__ uint32_t lds[];
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    uint32_t p = 17u;
    for (uint32_t i = 0; i < hops; i++) p = __builtin_nontemporal_load(nxt + p);
    lds[0] = p;
    out[1] = p;
}

struct Bar {
    uint32_t* flat;    // [0]: arrivals (monotonic)
    uint32_t* xcd;     // [8 * 32]: per-XCD arrivals, 128 bytes apart
    uint32_t* err;
};

// flat: every workgroup adds to one counter and waits for it to reach (r + 1) G
__device__ __forceinline__ void bar_flat(const Bar& b, uint32_t r) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t target = (r + 1) * gridDim.x;
        __hip_atomic_fetch_add(b.flat, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t s = 0;
        while (__hip_atomic_load(b.flat, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++s > kSpinMax) { atomicOr(b.err, 1u); break; }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

// two levels: the workgroups of one XCD (blockIdx % 8) count on their own line;
// the last of them adds 1 to the flat counter, which every workgroup waits on
__device__ __forceinline__ void bar_xcd(const Bar& b, uint32_t r) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t x = blockIdx.x & 7u, per = (gridDim.x - x + 7u) / 8u;
        const uint32_t old = __hip_atomic_fetch_add(b.xcd + 32 * x, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == (r + 1) * per) __hip_atomic_fetch_add(b.flat, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t target = (r + 1) * min(8u, gridDim.x);
        uint32_t s = 0;
        while (__hip_atomic_load(b.flat, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++s > kSpinMax) { atomicOr(b.err, 1u); break; }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

// `rounds` barriers in one launch; with `dirty`, every thread first stores one
// word at a pseudo-random slot of buf (so each barrier's release writes back
// dirty lines) and, after the barrier, reads one written by another workgroup
template <int kMode>
__global__ __launch_bounds__(kBlock) void k_persist(Bar b, uint32_t rounds, uint32_t* buf, uint32_t nbuf, uint32_t dirty,
                                                    uint32_t* out) {
    extern __shared__ uint32_t lds[];
    uint32_t acc = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        if (dirty) {
            const uint32_t i = (blockIdx.x * kBlock + threadIdx.x) * 2654435761u + r * 40503u;
            buf[i % nbuf] = r + 1;
        }
        if (kMode == 0) bar_flat(b, r); else bar_xcd(b, r);
        if (dirty) {
            const uint32_t i = ((blockIdx.x + 1) % gridDim.x * kBlock + threadIdx.x) * 2654435761u + r * 40503u;
            acc += buf[i % nbuf];
        }
    }
    lds[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0 && lds[1] == 0xFFFFFFFFu) out[0] = acc;
}

int main(int argc, char** argv) {
    const int reps = 200;
    const uint32_t lds = 24 * 1024;   // the ELL round kernel's dynamic LDS at W = 6
    int dev = 0, cus = 0;
    CHK(hipGetDevice(&dev));
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int occ = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_persist<0>, kBlock, lds));
    const uint32_t G = uint32_t(occ * cus);
    printf("CUs %d, resident workgroups of %d threads with %u B LDS: %d per CU, grid %u\n", cus, kBlock, lds, occ, G);

    const uint32_t nchain = 1u << 26;
    uint32_t *nxt, *out, *cnt, *buf;
    CHK(hipMalloc(&nxt, size_t(nchain) * 4));
    CHK(hipMalloc(&out, 64));
    CHK(hipMalloc(&cnt, 512));
    CHK(hipMemset(cnt, 0, 512));
    const uint32_t nbuf = 10u << 20;   // 40 MB
    CHK(hipMalloc(&buf, size_t(nbuf) * 4));
    CHK(hipMemset(buf, 0, size_t(nbuf) * 4));
    {
        std::vector<uint32_t> h(nchain);
        uint64_t x = 88172645463325252ull;
        for (uint32_t i = 0; i < nchain; i++) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            h[i] = uint32_t(x % nchain);   // every value < nchain: the chase stays in bounds
        }
        CHK(hipMemcpy(nxt, h.data(), size_t(nchain) * 4, hipMemcpyHostToDevice));
    }
    Bar b;
    CHK(hipMalloc(&b.flat, 4096));
    b.xcd = b.flat + 64;
    b.err = b.flat + 32;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    float ms = 0;

    auto launches = [&](const char* name, auto launch) -> int {
        for (int i = 0; i < 10; i++) launch();
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; i++) launch();
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-52s %8.2f us per launch\n", name, ms * 1000.f / reps);
        return 0;
    };
    if (launches("empty, grid 1", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(kBlock), lds, 0, out); })) return 1;
    if (launches("empty, grid 256", [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(kBlock), lds, 0, out); })) return 1;
    if (launches("empty, resident grid", [&] { hipLaunchKernelGGL(k_empty, dim3(G), dim3(kBlock), lds, 0, out); })) return 1;
    if (launches("empty, resident grid, no LDS", [&] { hipLaunchKernelGGL(k_empty, dim3(G), dim3(kBlock), 1024, 0, out); })) return 1;
    if (launches("counts read, resident grid", [&] { hipLaunchKernelGGL(k_counts, dim3(G), dim3(kBlock), lds, 0, cnt, out); })) return 1;
    for (uint32_t hops : {1u, 4u, 10u, 20u}) {
        char name[96];
        snprintf(name, sizeof name, "chain of %u dependent loads, resident grid", hops);
        if (launches(name, [&] { hipLaunchKernelGGL(k_chain, dim3(G), dim3(kBlock), lds, 0, nxt, hops, out); })) return 1;
    }
    for (uint32_t hops : {10u, 20u}) {
        char name[96];
        snprintf(name, sizeof name, "chain of %u dependent loads, grid 1", hops);
        if (launches(name, [&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(kBlock), lds, 0, nxt, hops, out); })) return 1;
    }

    // persistent: `R` barriers in one launch, normal and cooperative launch
    const uint32_t R = 200;
    for (int mode = 0; mode < 2; mode++)
        for (uint32_t dirty = 0; dirty < 2; dirty++)
            for (uint32_t g : {256u, G}) {
                for (int coop = 0; coop < 2; coop++) {
                    CHK(hipMemset(b.flat, 0, 4096));
                    CHK(hipDeviceSynchronize());
                    uint32_t rr = R;
                    void* args[] = {&b, &rr, &buf, (void*)&nbuf, &dirty, &out};
                    const void* fn = mode == 0 ? (const void*)k_persist<0> : (const void*)k_persist<1>;
                    CHK(hipEventRecord(e0, 0));
                    if (coop) {
                        const hipError_t e = hipLaunchCooperativeKernel(fn, dim3(g), dim3(kBlock), args, lds, 0);
                        if (e != hipSuccess) {
                            printf("cooperative launch of %u workgroups: %s\n", g, hipGetErrorString(e));
                            (void)hipGetLastError();
                            continue;
                        }
                    } else {
                        CHK(hipLaunchKernel(fn, dim3(g), dim3(kBlock), args, lds, 0));
                    }
                    CHK(hipEventRecord(e1, 0));
                    CHK(hipEventSynchronize(e1));
                    CHK(hipEventElapsedTime(&ms, e0, e1));
                    uint32_t hb[2];
                    CHK(hipMemcpy(hb, b.flat, 4, hipMemcpyDeviceToHost));
                    CHK(hipMemcpy(hb + 1, b.err, 4, hipMemcpyDeviceToHost));
                    printf("persistent %-4s barrier, grid %4u, %s, %-11s: %8.2f us per round (%u rounds, %.1f us launch total)%s\n",
                           mode == 0 ? "flat" : "xcd", g, dirty ? "dirty" : "clean", coop ? "cooperative" : "normal",
                           ms * 1000.f / R, R, ms * 1000.f, hb[1] ? "  SPIN LIMIT HIT" : "");
                }
            }
    CHK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
