// Host-only stand-in for <rccl/rccl.h>: the types and entry points
// rccl_comm.cpp uses, implemented by rccl_stub.cpp as a recorder so the
// plan building and argument checks run under ASan / UBSan without a GPU.
#pragma once
#include <cstddef>

#include "hip/hip_runtime.h"

typedef enum { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
               ncclInvalidArgument = 4, ncclInvalidUsage = 5, ncclRemoteError = 6 } ncclResult_t;
typedef enum { ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5,
               ncclFloat16 = 6, ncclFloat32 = 7, ncclFloat64 = 8 } ncclDataType_t;
typedef enum { ncclSum = 0, ncclProd = 1, ncclMax = 2, ncclMin = 3 } ncclRedOp_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef struct ncclComm* ncclComm_t;

extern "C" {
ncclResult_t ncclGetUniqueId(ncclUniqueId* id);
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank);
ncclResult_t ncclCommDestroy(ncclComm_t comm);
ncclResult_t ncclCommAbort(ncclComm_t comm);
ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* err);
ncclResult_t ncclCommCount(ncclComm_t comm, int* count);
const char* ncclGetErrorString(ncclResult_t r);
ncclResult_t ncclGroupStart();
ncclResult_t ncclGroupEnd();
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t s);
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t s);
ncclResult_t ncclAllReduce(const void* sb, void* rb, size_t count, ncclDataType_t dt, ncclRedOp_t op, ncclComm_t comm,
                           hipStream_t s);
ncclResult_t ncclBroadcast(const void* sb, void* rb, size_t count, ncclDataType_t dt, int root, ncclComm_t comm,
                           hipStream_t s);
}
