// Host-only stand-in for <hip/hip_runtime.h> in the RCCL plan sanitizer build
// (tests/test_native_sanitizers.py): rccl_comm.cpp only names hipStream_t.
#pragma once
typedef struct ihipStream_t* hipStream_t;
