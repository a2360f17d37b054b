// The part of the RCCL C API the native runtime uses, resolved at run time.
//
// Why not <rccl/rccl.h> + -lrccl: the library was compiled against the ROCm
// 7.2 headers (RCCL 2.27.7) but a process that imported PyTorch first runs
// PyTorch's bundled librccl.so.1 (2.26.6): same SONAME, so the dynamic linker
// binds every call to the copy already loaded, whatever the headers said
// (round-3 finding).  Declaring only the calls used here (communicator
// bootstrap, grouped send/recv, error strings) and resolving them with dlsym
// from the librccl.so.1 the process actually holds makes the binding explicit;
// rccl_api() then checks the loaded version against the range these
// declarations are valid for and refuses anything else loudly.
//
// Every declaration below is unchanged across RCCL 2.18 .. 2.27 (the NCCL 2
// API: ncclUniqueId is 128 bytes, ncclFloat32 = 7, ncclFloat64 = 8, the
// signatures of ncclSend / ncclRecv / ncclCommInitRank).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

typedef struct ncclComm* ncclComm_t;
#define NCCL_UNIQUE_ID_BYTES 128
typedef struct { char internal[NCCL_UNIQUE_ID_BYTES]; } ncclUniqueId;
typedef enum { ncclSuccess = 0 } ncclResult_t;
typedef enum { ncclFloat32 = 7, ncclFloat64 = 8 } ncclDataType_t;

// oldest / newest RCCL version code (major * 10000 + minor * 100 + patch)
// these declarations are checked against
#define STSP_RCCL_MIN_VERSION 21800
#define STSP_RCCL_MAX_VERSION 22999

struct RcclApi {
  ncclResult_t (*GetVersion)(int*);
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*);
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  const char* (*GetErrorString)(ncclResult_t);
  int version;          // ncclGetVersion of the loaded library (0: none)
  const char* path;     // where it was found
};

// The resolved API, or nullptr (then stsp_rccl_error() says why).
const RcclApi* rccl_api();
