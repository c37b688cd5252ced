// loopback_rccl.cpp -- TEST-ONLY stand-in for librccl.so.1 (never shipped,
// never on the product's search path).  It exports the nine RCCL symbols
// rt_multi / rt_comm resolve at run time (simd-ray-tracer_amd/csrc/rt_multi.cpp,
// rccl()) with RCCL's point-to-point semantics, so that rt_multi's RCCL branch
// -- grouped ncclSend/ncclRecv of every shard's band image, mean and ray count
// to devices[0], the transfer streams, the two-slot double buffering and the
// `sent` events -- runs on a one-GPU box, where the real RCCL refuses a device
// listed twice.  tests/conftest.py starts tests/loopback_rccl/multi_rccl_check
// with this directory first on LD_LIBRARY_PATH, before the test process
// touches the GPU; tests/test_gpu_multi.py checks its frames.
//
// Semantics kept from RCCL (rccl.h: ncclSend / ncclRecv, ncclGroupStart /
// ncclGroupEnd): operations posted inside a group are matched at the
// outermost ncclGroupEnd, a send of comm rank r to peer p with the first
// unmatched receive of comm rank p from peer r (same communicator clique,
// posting order), and the byte counts must agree.  A matched pair becomes
// one copy on the RECEIVER's stream after everything already enqueued on
// the SENDER's stream (an event), and the sender's stream then waits for the
// copy (a second event): a buffer handed to ncclSend may be overwritten by
// work enqueued on its stream after the group, exactly as with RCCL.  A send
// or receive left unmatched at ncclGroupEnd is ncclInvalidUsage.
//
// rtLoopbackSharedDevices marks this library: rt_multi_create then allows the
// RCCL transport over a device listed more than once (the real RCCL refuses
// such a communicator, so the product never tries it with the real one).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>
#include <vector>

struct ncclComm {
    int rank = 0, nranks = 1, dev = 0;
    int clique = 0;
};

namespace {

struct Op {
    bool send;
    ncclComm_t comm;
    int peer;
    void *buf;
    size_t bytes;
    hipStream_t stream;
    bool matched;
};

thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;
std::mutex g_mu;
int g_next_clique = 1;

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

struct DeviceRestore {
    int dev = 0;
    DeviceRestore() { (void)hipGetDevice(&dev); }
    ~DeviceRestore() { (void)hipSetDevice(dev); }
};

// one matched send -> recv pair: copy on the receiver's stream, ordered after the sender's stream,
// and the sender's stream ordered after the copy
ncclResult_t transfer(const Op &s, const Op &r) {
    hipEvent_t sent = nullptr, copied = nullptr;
    if (hipSetDevice(s.comm->dev) != hipSuccess ||
        hipEventCreateWithFlags(&sent, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(sent, s.stream) != hipSuccess)
        return ncclUnhandledCudaError;
    if (hipSetDevice(r.comm->dev) != hipSuccess || hipStreamWaitEvent(r.stream, sent, 0) != hipSuccess)
        return ncclUnhandledCudaError;
    const hipError_t e = s.comm->dev == r.comm->dev
                             ? hipMemcpyAsync(r.buf, s.buf, s.bytes, hipMemcpyDeviceToDevice, r.stream)
                             : hipMemcpyPeerAsync(r.buf, r.comm->dev, s.buf, s.comm->dev, s.bytes, r.stream);
    if (e != hipSuccess || hipEventCreateWithFlags(&copied, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(copied, r.stream) != hipSuccess)
        return ncclUnhandledCudaError;
    if (hipSetDevice(s.comm->dev) != hipSuccess || hipStreamWaitEvent(s.stream, copied, 0) != hipSuccess)
        return ncclUnhandledCudaError;
    (void)hipEventDestroy(sent);  // released once the recorded work completes
    (void)hipEventDestroy(copied);
    return ncclSuccess;
}

ncclResult_t flush() {
    DeviceRestore restore;
    std::vector<Op> ops;
    ops.swap(g_ops);
    for (Op &s : ops) {
        if (!s.send) continue;
        Op *r = nullptr;
        for (Op &c : ops)
            if (!c.send && !c.matched && c.comm->clique == s.comm->clique && c.comm->rank == s.peer &&
                c.peer == s.comm->rank) {
                r = &c;
                break;
            }
        if (!r || r->bytes != s.bytes) return ncclInvalidUsage;
        r->matched = s.matched = true;
        if (s.bytes)
            if (const ncclResult_t rc = transfer(s, *r)) return rc;
    }
    for (const Op &o : ops)
        if (!o.matched) return ncclInvalidUsage;
    return ncclSuccess;
}

ncclResult_t post(bool send, const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                  hipStream_t stream) {
    const size_t tb = type_bytes(t);
    if (!comm || tb == 0 || peer < 0 || peer >= comm->nranks || (count && !buf)) return ncclInvalidArgument;
    g_ops.push_back({send, comm, peer, const_cast<void *>(buf), count * tb, stream, false});
    return g_depth == 0 ? flush() : ncclSuccess;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) int rtLoopbackSharedDevices = 1;

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    if (!id) return ncclInvalidArgument;
    memset(id, 0, sizeof(*id));
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t *comms, int ndev, const int *devlist) {
    if (!comms || ndev <= 0) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lock(g_mu);
    const int clique = g_next_clique++;
    for (int i = 0; i < ndev; ++i) {
        comms[i] = new ncclComm();
        comms[i]->rank = i;
        comms[i]->nranks = ndev;
        comms[i]->dev = devlist ? devlist[i] : i;
        comms[i]->clique = clique;
    }
    return ncclSuccess;
}

// one-process-per-GPU communicators cannot meet inside one loopback process: a
// communicator of one rank only (rt_comm's self-gather)
ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId, int rank) {
    if (!comm || nranks != 1 || rank != 0) return ncclInvalidUsage;
    std::lock_guard<std::mutex> lock(g_mu);
    *comm = new ncclComm();
    (void)hipGetDevice(&(*comm)->dev);
    (*comm)->clique = g_next_clique++;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

ncclResult_t ncclSend(const void *sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return post(true, sendbuff, count, datatype, peer, comm, stream);
}

ncclResult_t ncclRecv(void *recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return post(false, recvbuff, count, datatype, peer, comm, stream);
}

ncclResult_t ncclGroupStart() {
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_depth == 0) return ncclInvalidUsage;
    return --g_depth == 0 ? flush() : ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t result) {
    switch (result) {
        case ncclSuccess: return "no error (loopback)";
        case ncclInvalidArgument: return "invalid argument (loopback)";
        case ncclInvalidUsage: return "invalid usage: unmatched send/recv (loopback)";
        default: return "HIP error (loopback)";
    }
}

}  // extern "C"
