// socket_net.h — the p2p net the SwitchML plugin library gives RCCL.
//
// NCCL/RCCL take a CollNet table only from a library whose net table works
// (the net and CollNet of one library are a pair; a failed net init or zero
// net devices drops both).  The reference gets its net by patching NCCL to
// hand its internal IB net to the plugin (switchml_nccl.patch:24-81); RCCL
// 7.2 cannot be patched here, so the library carries its own: a TCP net over
// the ncclNet_v6 contract —
//   * listen() binds a socket and writes {magic, IPv4 address, port, nonce}
//     into the 128-byte handle RCCL passes to the peer through its bootstrap;
//   * connect() / accept() are non-blocking in the v5+ sense: they may return
//     a NULL comm and RCCL calls again;
//   * isend / irecv post requests that test() progresses over a non-blocking
//     socket, FIFO per comm (what NCCL's matching of sends to receives on one
//     connection assumes); every message carries an 8-byte {size, tag}
//     header, so a receive learns the size the sender posted;
//   * host memory only (ptrSupport = NCCL_PTR_HOST): RCCL stages device data
//     through its host proxy buffers.
// Address: SWITCHML_NET_IFADDR (dotted IPv4), else the first UP non-loopback
// IPv4 interface whose name starts with SWITCHML_NET_IFNAME (any name when
// unset), else 127.0.0.1.
#ifndef SWITCHML_AMD_SOCKET_NET_H_
#define SWITCHML_AMD_SOCKET_NET_H_

#include "collnet_abi.h"

namespace sml_net {

ncclResult_t Init(ncclDebugLogger_t logger);
ncclResult_t Devices(int* ndev);
ncclResult_t GetProperties(int dev, ncclNetProperties_v6_t* props);
ncclResult_t Listen(int dev, void* handle, void** listen_comm);
ncclResult_t Connect(int dev, void* handle, void** send_comm);
ncclResult_t Accept(void* listen_comm, void** recv_comm);
ncclResult_t RegMr(void* comm, void* data, int size, int type, void** mhandle);
ncclResult_t RegMrDmaBuf(void* comm, void* data, size_t size, int type, uint64_t offset, int fd, void** mhandle);
ncclResult_t DeregMr(void* comm, void* mhandle);
ncclResult_t Isend(void* send_comm, void* data, int size, int tag, void* mhandle, void** request);
ncclResult_t Irecv(void* recv_comm, int n, void** data, int* sizes, int* tags, void** mhandles, void** request);
ncclResult_t Iflush(void* recv_comm, int n, void** data, int* sizes, void** mhandles, void** request);
ncclResult_t Test(void* request, int* done, int* sizes);
ncclResult_t CloseSend(void* send_comm);
ncclResult_t CloseRecv(void* recv_comm);
ncclResult_t CloseListen(void* listen_comm);

}  // namespace sml_net

#endif  // SWITCHML_AMD_SOCKET_NET_H_
