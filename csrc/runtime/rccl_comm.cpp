// Native RCCL communicator for the frame-level data-parallel exchange.
//
// torch.distributed's batch_isend_irecv builds one P2POp object per tensor,
// enters ncclGroupStart/End through Python, and records a work handle per op.
// The DP exchange moves a handful of fixed-shape buffers per step, so the
// Python side is most of its latency at small (detection-sized) payloads.
// This file owns a second RCCL communicator (same ranks, bootstrapped from a
// unique id that rank 0 broadcasts over the process group) and issues a whole
// scatter / gather plan as ONE ncclGroupStart .. ncclGroupEnd from C++ on the
// caller's HIP stream — no host sync, capturable into a hipGraph like any
// other stream work.  xGMI is point-to-point, so a grouped fan-out drives
// every link at once (parallel/dp.py module docstring).
//
// Reference parity: the reference has no multi-GPU path at all (SURVEY §2.5,
// §5.8); this is the native runtime under parallel/rccl.py.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>

extern "C" {

// 128-byte opaque bootstrap id (rank 0 creates it, the process group spreads it)
int tca_rccl_unique_id_bytes() { return (int)sizeof(ncclUniqueId); }

int tca_rccl_get_unique_id(void* out) {
    if (!out) return (int)ncclInvalidArgument;
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return (int)r;
    std::memcpy(out, &id, sizeof(id));
    return 0;
}

// comm_out receives the ncclComm_t handle.  The caller has already selected
// its HIP device (torch.cuda.set_device).
int tca_rccl_comm_init(void** comm_out, int nranks, const void* id_bytes, int rank) {
    if (!comm_out || !id_bytes || nranks < 1 || rank < 0 || rank >= nranks) return (int)ncclInvalidArgument;
    *comm_out = nullptr;
    ncclUniqueId id;
    std::memcpy(&id, id_bytes, sizeof(id));
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
    *comm_out = (void*)comm;
    return (int)r;
}

int tca_rccl_comm_destroy(void* comm) { return comm ? (int)ncclCommDestroy((ncclComm_t)comm) : 0; }

// tear down without waiting for outstanding work (a peer died mid-step)
int tca_rccl_comm_abort(void* comm) { return comm ? (int)ncclCommAbort((ncclComm_t)comm) : 0; }

int tca_rccl_async_error(void* comm) {
    if (!comm) return (int)ncclInvalidArgument;
    ncclResult_t e = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError((ncclComm_t)comm, &e);
    return r != ncclSuccess ? (int)r : (int)e;
}

// Ranks the communicator was built over (ncclCommCount): what the bench reports as n_gpus.
int tca_rccl_comm_count(void* comm, int* count) {
  if (!comm || !count) return (int)ncclInvalidArgument;
  return (int)ncclCommCount((ncclComm_t)comm, count);
}

const char* tca_rccl_error_string(int code) { return ncclGetErrorString((ncclResult_t)code); }

// One grouped p2p plan: n ops; op i moves bytes[i] bytes of buf[i] to
// (kind[i] = 0, send) or from (kind[i] = 1, recv) rank peer[i].  Payloads go
// as 4-byte words when size and alignment allow, bytes otherwise, so any
// dtype travels unchanged.  The whole plan is checked before the group opens
// (kind 0/1, peer inside the communicator, a buffer for every non-empty op),
// so a bad plan posts nothing and leaves no half-issued group behind.
int tca_rccl_group_p2p(void* comm, int n, const int* kind, const int* peer, void* const* buf,
                       const int64_t* bytes, void* stream) {
    ncclComm_t c = (ncclComm_t)comm;
    hipStream_t s = (hipStream_t)stream;
    if (!c || n < 0) return (int)ncclInvalidArgument;
    if (n > 0 && (!kind || !peer || !buf || !bytes)) return (int)ncclInvalidArgument;
    int nranks = 0;
    ncclResult_t r = ncclCommCount(c, &nranks);
    if (r != ncclSuccess) return (int)r;
    for (int i = 0; i < n; ++i) {
        if (kind[i] != 0 && kind[i] != 1) return (int)ncclInvalidArgument;
        if (bytes[i] > 0 && (peer[i] < 0 || peer[i] >= nranks || !buf[i])) return (int)ncclInvalidArgument;
    }
    r = ncclGroupStart();
    if (r != ncclSuccess) return (int)r;
    for (int i = 0; i < n && r == ncclSuccess; ++i) {
        const int64_t b = bytes[i];
        if (b <= 0) continue;
        const bool words = (b % 4 == 0) && ((uintptr_t)buf[i] % 4 == 0);
        const size_t cnt = words ? (size_t)(b / 4) : (size_t)b;
        const ncclDataType_t dt = words ? ncclInt32 : ncclUint8;
        r = kind[i] == 0 ? ncclSend(buf[i], cnt, dt, peer[i], c, s) : ncclRecv(buf[i], cnt, dt, peer[i], c, s);
    }
    ncclResult_t e = ncclGroupEnd();
    return r != ncclSuccess ? (int)r : (int)e;
}

// in-place MAX all-reduce of n doubles (step-time aggregation in bench.py)
int tca_rccl_allreduce_max_f64(void* comm, double* buf, int64_t n, void* stream) {
    if (!comm || n < 0 || (n > 0 && !buf)) return (int)ncclInvalidArgument;
    return (int)ncclAllReduce(buf, buf, (size_t)n, ncclFloat64, ncclMax, (ncclComm_t)comm, (hipStream_t)stream);
}

// in-place broadcast of nbytes from root (parameter broadcast for DP replicas)
int tca_rccl_broadcast(void* comm, void* buf, int64_t nbytes, int root, void* stream) {
    int nranks = 0;
    if (!comm || nbytes < 0 || (nbytes > 0 && !buf)) return (int)ncclInvalidArgument;
    if (ncclCommCount((ncclComm_t)comm, &nranks) != ncclSuccess || root < 0 || root >= nranks)
        return (int)ncclInvalidArgument;
    return (int)ncclBroadcast(buf, buf, (size_t)nbytes, ncclUint8, root, (ncclComm_t)comm, (hipStream_t)stream);
}

}  // extern "C"
