// Microtest of the per-wave LDS send buffer (psim_internal.h WaveQ): every
// thread sends a data-dependent number of records from divergent code; the
// host checks that each (sender, index) record lands exactly once.
#include "../../partisan_amd/csrc/psim_internal.h"
#include <cstdio>
#include <vector>

using namespace psim;
struct Rec { uint32_t type, src, dst, seq, a, b; };

__device__ __forceinline__ uint32_t mix(uint32_t x) { x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; return x ^ (x >> 16); }

__device__ void send(WaveQ<Rec> q, uint32_t* cnt, Rec* out, uint32_t cap, uint32_t& err, uint32_t v, uint32_t& seq, uint32_t kind) {
    wq_send(q, cnt, out, cap, err, Rec{kind, v, 0, seq++, 0, 0});
}

__global__ __launch_bounds__(256) void k_wq(Rec* out, uint32_t* cnt, uint32_t cap, uint32_t n, uint32_t* errs) {
    __shared__ Rec qb[4][kWq];
    __shared__ uint32_t qn[4];
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    const WaveQ<Rec> q{qb[threadIdx.x >> 6], &qn[threadIdx.x >> 6]};
    wq_init(q.n);
    uint32_t err = 0, seq = 0;
    if (v < n) {
        const uint32_t h = mix(v);
        const uint32_t a = h % 9, b = (h >> 8) % 5;
        for (uint32_t i = 0; i < a; i++) {
            if ((h >> i) & 1) send(q, cnt, out, cap, err, v, seq, 1);
            else {
                send(q, cnt, out, cap, err, v, seq, 2);
                if (i & 1) send(q, cnt, out, cap, err, v, seq, 3);
            }
        }
        if (h & 0x10000) for (uint32_t i = 0; i < b * 10; i++) send(q, cnt, out, cap, err, v, seq, 4);
    }
    wq_flush(q, cnt, out, cap, err);
    if (err) atomicOr(errs, err);
}

int main() {
    const uint32_t n = 1u << 20, cap = 40u * n;
    Rec* out; uint32_t *cnt, *errs;
    hipMalloc(&out, size_t(cap) * sizeof(Rec));
    hipMalloc(&cnt, 4); hipMalloc(&errs, 4);
    hipMemset(cnt, 0, 4); hipMemset(errs, 0, 4);
    hipMemset(out, 0xFF, size_t(cap) * sizeof(Rec));
    hipLaunchKernelGGL(k_wq, dim3((n + 255) / 256), dim3(256), 0, 0, out, cnt, cap, n, errs);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
    uint32_t c = 0, e = 0;
    hipMemcpy(&c, cnt, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&e, errs, 4, hipMemcpyDeviceToHost);
    std::vector<Rec> h(c < cap ? c : cap);
    hipMemcpy(h.data(), out, h.size() * sizeof(Rec), hipMemcpyDeviceToHost);
    // expected per sender: the same walk on the host
    std::vector<uint32_t> want(n), got(n, 0);
    uint64_t total = 0;
    auto mixh = [](uint32_t x) { x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; return x ^ (x >> 16); };
    for (uint32_t v = 0; v < n; v++) {
        const uint32_t hh = mixh(v), a = hh % 9, b = (hh >> 8) % 5;
        uint32_t s = 0;
        for (uint32_t i = 0; i < a; i++) s += ((hh >> i) & 1) ? 1 : ((i & 1) ? 2 : 1);
        if (hh & 0x10000) s += b * 10;
        want[v] = s; total += s;
    }
    uint64_t bad = 0;
    std::vector<uint64_t> seen(n, 0);
    for (const Rec& r : h) {
        if (r.src >= n || r.seq >= 64) { bad++; continue; }
        if (seen[r.src] >> r.seq & 1) bad++;
        seen[r.src] |= 1ull << r.seq;
        got[r.src]++;
    }
    uint64_t miss = 0;
    for (uint32_t v = 0; v < n; v++) if (got[v] != want[v]) miss++;
    printf("records %u expected %llu err %u bad %llu senders_wrong %llu\n", c, (unsigned long long)total, e,
           (unsigned long long)bad, (unsigned long long)miss);
    return (c == total && !bad && !miss && !e) ? 0 : 1;
}
