// transport.hip -- the cross-shard exchange of a vertex-sharded handle, inside
// libpsim ("multi-GPU handles own ... one RCCL communicator";
// 8(e)).  One process per GPU; the library owns the communicator and moves
// every round's cross-shard inbox words itself, stream-ordered after the round
// kernel's pack and before the ingest, so a whole heartbeat (psim_shard_run)
// runs with one host synchronisation per 4-round chunk.
//
//   * RcclTransport: ncclCommInitRank on the handle's device from a unique id
//     the caller distributes; the words move as ONE grouped set of
//     ncclSend / ncclRecv per round (an all-to-all-v with the static region
//     sizes of psim_shard_layout / psim_shard_recv_layout: xGMI is point to
//     point, every peer pair is its own transfer, no ring); the per-chunk
//     counters are one int64 ncclAllReduce.
//   * CallbackTransport: a caller-supplied psim_transport (tests: gloo from
//     Python) over host staging buffers.
#include "psim_internal.h"
#include "../../include/psim.h"

#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

namespace psim {

namespace {

class RcclTransport : public Transport {
  public:
    ncclComm_t comm = nullptr;
    int64_t* dbuf = nullptr;          // device scratch for the counter all-reduce
    size_t dcap = 0;
    std::string err;

    ~RcclTransport() override {
        if (dbuf) (void)hipFree(dbuf);
        if (comm) (void)ncclCommDestroy(comm);
    }

    int fail_nccl(ncclResult_t r, const char* what, std::string* e) {
        if (e) *e = std::string(what) + ": " + ncclGetErrorString(r);
        return PSIM_ERCCL;
    }

    int alltoallv(const uint32_t* send, const uint64_t* soff, uint32_t* recv, const uint64_t* roff, int rank, int world,
                  hipStream_t s, std::string* e) override {
        ncclResult_t r = ncclGroupStart();
        if (r != ncclSuccess) return fail_nccl(r, "ncclGroupStart", e);
        for (int d = 0; d < world; d++) {
            if (d == rank) continue;
            const size_t ns = size_t(soff[d + 1] - soff[d]), nr = size_t(roff[d + 1] - roff[d]);
            if (ns) {
                r = ncclSend(send + soff[d], ns, ncclUint32, d, comm, s);
                if (r != ncclSuccess) { (void)ncclGroupEnd(); return fail_nccl(r, "ncclSend", e); }
            }
            if (nr) {
                r = ncclRecv(recv + roff[d], nr, ncclUint32, d, comm, s);
                if (r != ncclSuccess) { (void)ncclGroupEnd(); return fail_nccl(r, "ncclRecv", e); }
            }
        }
        r = ncclGroupEnd();
        return r == ncclSuccess ? PSIM_OK : fail_nccl(r, "ncclGroupEnd", e);
    }

    int allreduce(int64_t* vals, size_t n, hipStream_t s, std::string* e) override {
        if (!n) return PSIM_OK;
        if (n > dcap) {
            if (dbuf) (void)hipFree(dbuf);
            dbuf = nullptr;
            dcap = 0;
            if (hipMalloc((void**)&dbuf, n * sizeof(int64_t)) != hipSuccess) {
                if (e) *e = "counter all-reduce buffer";
                return PSIM_ENOMEM;
            }
            dcap = n;
        }
        if (hipMemcpyAsync(dbuf, vals, n * 8, hipMemcpyHostToDevice, s) != hipSuccess) return PSIM_EHIP;
        const ncclResult_t r = ncclAllReduce(dbuf, dbuf, n, ncclInt64, ncclSum, comm, s);
        if (r != ncclSuccess) return fail_nccl(r, "ncclAllReduce", e);
        if (hipMemcpyAsync(vals, dbuf, n * 8, hipMemcpyDeviceToHost, s) != hipSuccess) return PSIM_EHIP;
        return hipStreamSynchronize(s) == hipSuccess ? PSIM_OK : PSIM_EHIP;
    }

    int allgather(uint32_t* buf, size_t count, int rank, int world, hipStream_t s, std::string* e) override {
        (void)world;
        if (!count) return PSIM_OK;
        const ncclResult_t r = ncclAllGather(buf + size_t(rank) * count, buf, count, ncclUint32, comm, s);
        return r == ncclSuccess ? PSIM_OK : fail_nccl(r, "ncclAllGather", e);
    }

    const char* name() const override { return "rccl"; }
    int comm_size() const override {
        int c = -1;
        return comm && ncclCommCount(comm, &c) == ncclSuccess ? c : -1;
    }
    int comm_rank() const override {
        int r = -1;
        return comm && ncclCommUserRank(comm, &r) == ncclSuccess ? r : -1;
    }
};

class CallbackTransport : public Transport {
  public:
    psim_transport t{};
    std::vector<uint32_t> hs, hr;      // host staging

    int alltoallv(const uint32_t* send, const uint64_t* soff, uint32_t* recv, const uint64_t* roff, int rank, int world,
                  hipStream_t s, std::string* e) override {
        (void)rank;
        hs.resize(size_t(soff[world]) + 1);
        hr.resize(size_t(roff[world]) + 1);
        if (soff[world] && hipMemcpyAsync(hs.data(), send, soff[world] * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
            return PSIM_EHIP;
        if (hipStreamSynchronize(s) != hipSuccess) return PSIM_EHIP;
        const int rc = t.alltoallv(t.ctx, hs.data(), soff, hr.data(), roff, world);
        if (rc) {
            if (e) *e = "psim_transport.alltoallv returned " + std::to_string(rc);
            return PSIM_ERCCL;
        }
        if (roff[world] && hipMemcpyAsync(recv, hr.data(), roff[world] * 4, hipMemcpyHostToDevice, s) != hipSuccess)
            return PSIM_EHIP;
        return hipStreamSynchronize(s) == hipSuccess ? PSIM_OK : PSIM_EHIP;
    }

    int allreduce(int64_t* vals, size_t n, hipStream_t s, std::string* e) override {
        (void)s;
        const int rc = t.allreduce(t.ctx, vals, n);
        if (rc && e) *e = "psim_transport.allreduce returned " + std::to_string(rc);
        return rc ? PSIM_ERCCL : PSIM_OK;
    }

    // through the caller's all-to-all-v: the own slice to every rank (host staged)
    int allgather(uint32_t* buf, size_t count, int rank, int world, hipStream_t s, std::string* e) override {
        if (!count) return PSIM_OK;
        const size_t tot = size_t(world) * count;
        hs.resize(tot + 1);
        hr.resize(tot + 1);
        if (hipMemcpyAsync(hs.data(), buf + size_t(rank) * count, count * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return PSIM_EHIP;
        for (int d = 1; d < world; d++) memcpy(hs.data() + size_t(d) * count, hs.data(), count * 4);
        std::vector<uint64_t> off(world + 1);
        for (int d = 0; d <= world; d++) off[d] = uint64_t(d) * count;
        const int rc = t.alltoallv(t.ctx, hs.data(), off.data(), hr.data(), off.data(), world);
        if (rc) {
            if (e) *e = "psim_transport.alltoallv (allgather) returned " + std::to_string(rc);
            return PSIM_ERCCL;
        }
        memcpy(hr.data() + size_t(rank) * count, hs.data(), count * 4);
        if (hipMemcpyAsync(buf, hr.data(), tot * 4, hipMemcpyHostToDevice, s) != hipSuccess) return PSIM_EHIP;
        return hipStreamSynchronize(s) == hipSuccess ? PSIM_OK : PSIM_EHIP;
    }

    const char* name() const override { return "callback"; }
};

}  // namespace

int make_rccl_transport(int device, int rank, int world, const void* id, Transport** out, std::string* err) {
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return PSIM_EHIP;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    auto* t = new (std::nothrow) RcclTransport();
    if (!t) return PSIM_ENOMEM;
    const ncclResult_t r = ncclCommInitRank(&t->comm, world, uid, rank);
    if (r != ncclSuccess) {
        if (err) *err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        t->comm = nullptr;
        delete t;
        return PSIM_ERCCL;
    }
    *out = t;
    return PSIM_OK;
}

Transport* make_callback_transport(const psim_transport& t) {
    auto* c = new (std::nothrow) CallbackTransport();
    if (c) c->t = t;
    return c;
}

int rccl_unique_id(void* out) {
    ncclUniqueId uid;
    const ncclResult_t r = ncclGetUniqueId(&uid);
    if (r != ncclSuccess) return PSIM_ERCCL;
    memcpy(out, &uid, sizeof uid);
    return PSIM_OK;
}

}  // namespace psim
