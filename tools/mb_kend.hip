// mb_kend.hip -- the kernel boundary of a round that stored something: per
// launch time of the resident grid when the launch stores K random 4-byte
// words (K = 0 .. 4M) into a 200 MB buffer, by store flavour (plain, non-
// temporal, system-scope relaxed atomic store), and the same with the next
// launch reading back the words the last one stored (the sparse rounds'
// pattern: round R's words are round R+1's inbox).  What a sparse Plumtree
// round pays at its end for the L2 write-back of its few dirty lines.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mb_kend.hip -o /tmp/mb_kend
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t slot(uint32_t i, uint32_t salt, uint32_t nbuf) {
    uint32_t x = i * 2654435761u + salt * 40503u;
    x ^= x >> 15;
    return (x * 2246822519u) % nbuf;
}

// kMode 0 plain store, 1 non-temporal store, 2 relaxed system-scope atomic store
template <int kMode>
__global__ __launch_bounds__(kBlock) void k_store(uint32_t* buf, uint32_t nbuf, uint32_t k, uint32_t salt,
                                                  uint32_t rd, uint32_t* out) {
    extern __shared__ uint32_t lds[];
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x, G = gridDim.x * kBlock;
    uint32_t acc = 0;
    for (uint32_t i = g; i < k; i += G) {
        if (rd) acc += buf[slot(i, salt - 1u, nbuf)];   // the words the last launch stored
        uint32_t* p = buf + slot(i, salt, nbuf);
        if constexpr (kMode == 0) *p = salt + acc;
        else if constexpr (kMode == 1) __builtin_nontemporal_store(salt + acc, p);
        else __hip_atomic_store(p, salt + acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    lds[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0 && lds[1] == 0xFFFFFFFFu) out[0] = acc;
}

int main() {
    const int reps = 100;
    const uint32_t lds = 24 * 1024;
    int dev = 0, cus = 0, occ = 0;
    CHK(hipGetDevice(&dev));
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_store<0>, kBlock, lds));
    const uint32_t G = uint32_t(occ * cus);
    printf("CUs %d, resident grid %u workgroups\n", cus, G);
    const uint32_t nbuf = 50u << 20;   // 200 MB: the 10M-vertex inbox
    uint32_t *buf, *out;
    CHK(hipMalloc(&buf, size_t(nbuf) * 4));
    CHK(hipMalloc(&out, 64));
    CHK(hipMemset(buf, 0, size_t(nbuf) * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const char* names[3] = {"plain", "nontemporal", "atomic-sys"};
    for (uint32_t rd = 0; rd < 2; rd++)
        for (int mode = 0; mode < 3; mode++)
            for (uint32_t k : {0u, 64u, 1024u, 16384u, 262144u, 4194304u}) {
                uint32_t salt = 1;
                auto launch = [&]() {
                    salt++;
                    if (mode == 0) hipLaunchKernelGGL(k_store<0>, dim3(G), dim3(kBlock), lds, 0, buf, nbuf, k, salt, rd, out);
                    else if (mode == 1) hipLaunchKernelGGL(k_store<1>, dim3(G), dim3(kBlock), lds, 0, buf, nbuf, k, salt, rd, out);
                    else hipLaunchKernelGGL(k_store<2>, dim3(G), dim3(kBlock), lds, 0, buf, nbuf, k, salt, rd, out);
                };
                for (int i = 0; i < 10; i++) launch();
                CHK(hipDeviceSynchronize());
                CHK(hipEventRecord(e0, 0));
                for (int i = 0; i < reps; i++) launch();
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                float ms = 0;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                printf("%-12s %s %8u words: %8.2f us per launch\n", names[mode], rd ? "read+store" : "store     ", k,
                       ms * 1000.f / reps);
            }
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
