// collnet_abi.h — the NCCL/RCCL CollNet plugin ABI, version 6.
//
// RCCL 7.2 loads "ncclCollNetPlugin_v6" .. "_v10" from the library named by
// NCCL_NET_PLUGIN (strings in /opt/rocm/lib/librccl.so), but its ext-net
// headers (net_v*.h) are not installed in this image.  The v6 layout below is
// restated from NCCL's published ext-net example headers (nccl/net_v6.h:
// ncclNetProperties_v6_t, ncclCollNet_v6_t) and the public enums of nccl.h.
// Only v6 is exported (CollNet and net tables): it is the oldest layout RCCL
// 7.2 accepts and the one whose field list is certain without the headers.
#ifndef SWITCHML_AMD_COLLNET_ABI_H_
#define SWITCHML_AMD_COLLNET_ABI_H_

#include <stddef.h>
#include <stdint.h>

extern "C" {

typedef enum {
    ncclSuccess = 0,
    ncclUnhandledCudaError = 1,
    ncclSystemError = 2,
    ncclInternalError = 3,
    ncclInvalidArgument = 4,
    ncclInvalidUsage = 5,
    ncclRemoteError = 6,
    ncclInProgress = 7
} ncclResult_t;

typedef enum {
    ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5,
    ncclFloat16 = 6, ncclFloat32 = 7, ncclFloat64 = 8, ncclBfloat16 = 9
} ncclDataType_t;

typedef enum { ncclSum = 0, ncclProd = 1, ncclMax = 2, ncclMin = 3, ncclAvg = 4 } ncclRedOp_t;

typedef enum { NCCL_LOG_NONE = 0, NCCL_LOG_VERSION = 1, NCCL_LOG_WARN = 2, NCCL_LOG_INFO = 3,
               NCCL_LOG_ABORT = 4, NCCL_LOG_TRACE = 5 } ncclDebugLogLevel;
typedef void (*ncclDebugLogger_t)(ncclDebugLogLevel level, unsigned long flags, const char* file, int line,
                                  const char* fmt, ...);

#define NCCL_PTR_HOST 0x1
#define NCCL_PTR_CUDA 0x2
#define NCCL_NET_HANDLE_MAXSIZE 128

typedef struct {
    char* name;
    char* pciPath;
    uint64_t guid;
    int ptrSupport;
    int speed;      // Mbps
    int port;
    float latency;
    int maxComms;
    int maxRecvs;
} ncclNetProperties_v6_t;

typedef struct {
    const char* name;
    ncclResult_t (*init)(ncclDebugLogger_t logFunction);
    ncclResult_t (*devices)(int* ndev);
    ncclResult_t (*getProperties)(int dev, ncclNetProperties_v6_t* props);
    ncclResult_t (*listen)(int dev, void* handle, void** listenComm);
    ncclResult_t (*connect)(void* handles[], int nranks, int rank, void* listenComm, void** collComm);
    ncclResult_t (*reduceSupport)(ncclDataType_t dataType, ncclRedOp_t redOp, int* supported);
    ncclResult_t (*regMr)(void* collComm, void* data, int size, int type, void** mhandle);
    ncclResult_t (*regMrDmaBuf)(void* collComm, void* data, size_t size, int type, uint64_t offset, int fd,
                                void** mhandle);
    ncclResult_t (*deregMr)(void* collComm, void* mhandle);
    ncclResult_t (*iallreduce)(void* collComm, void* sendData, void* recvData, int count, ncclDataType_t dataType,
                               ncclRedOp_t redOp, void* sendMhandle, void* recvMhandle, void** request);
    ncclResult_t (*iflush)(void* collComm, void* data, int size, void* mhandle, void** request);
    ncclResult_t (*test)(void* request, int* done, int* size);
    ncclResult_t (*closeColl)(void* collComm);
    ncclResult_t (*closeListen)(void* listenComm);
} ncclCollNet_v6_t;

// The p2p net table (nccl/net_v6.h ncclNet_v6_t).  The reference plugin
// exports one beside its CollNet table (switchml_plugin.cc:37: NCCL_PLUGIN_SYMBOL)
// and NCCL's loader looks the CollNet table up only in a library that has
// one; the SwitchML net table forwards to an underlying net plugin.
typedef struct {
    const char* name;
    ncclResult_t (*init)(ncclDebugLogger_t logFunction);
    ncclResult_t (*devices)(int* ndev);
    ncclResult_t (*getProperties)(int dev, ncclNetProperties_v6_t* props);
    ncclResult_t (*listen)(int dev, void* handle, void** listenComm);
    ncclResult_t (*connect)(int dev, void* handle, void** sendComm);
    ncclResult_t (*accept)(void* listenComm, void** recvComm);
    ncclResult_t (*regMr)(void* comm, void* data, int size, int type, void** mhandle);
    ncclResult_t (*regMrDmaBuf)(void* comm, void* data, size_t size, int type, uint64_t offset, int fd,
                                void** mhandle);
    ncclResult_t (*deregMr)(void* comm, void* mhandle);
    ncclResult_t (*isend)(void* sendComm, void* data, int size, int tag, void* mhandle, void** request);
    ncclResult_t (*irecv)(void* recvComm, int n, void** data, int* sizes, int* tags, void** mhandles,
                          void** request);
    ncclResult_t (*iflush)(void* recvComm, int n, void** data, int* sizes, void** mhandles, void** request);
    ncclResult_t (*test)(void* request, int* done, int* sizes);
    ncclResult_t (*closeSend)(void* sendComm);
    ncclResult_t (*closeRecv)(void* recvComm);
    ncclResult_t (*closeListen)(void* listenComm);
} ncclNet_v6_t;

}  // extern "C"

#endif  // SWITCHML_AMD_COLLNET_ABI_H_
