// switchml_collnet.cc — SwitchML as an RCCL CollNet plugin on MI355X
// (the reference's frameworks_integration/nccl_plugin/
// switchml_plugin.cc, rebuilt for the v6 plugin ABI RCCL 7.2 loads).
//
// RCCL hands a CollNet all-reduce to iallreduce(); the plugin submits it to
// the SwitchML Context (AllReduceAsync) and test() polls the Job, exactly as
// switchml_plugin.cc:293-387 does.  Differences, all deliberate:
//  * ptrSupport = NCCL_PTR_HOST | NCCL_PTR_CUDA (the reference: HOST only,
//    with "TODO | NCCL_PTR_CUDA" at :161) — device buffers go straight to the
//    GPU quantizer, no bounce copy;
//  * no p2p side channel: the reference forwarded listen/connect to NCCL's
//    internal IB net (:179-237) only to hold a ring neighbour it never used
//    for data; the switch (here: the Context's backend) does the reduction;
//  * a FAILED job makes test() return ncclInternalError (the reference kept
//    reporting "not done");
//  * ncclUint8 is widened to int32 as in :318-337 and narrowed back in
//    test() as in :370-378 — on the host for host buffers, by two small HIP
//    kernels into / out of a device int32 scratch for device buffers (the
//    reference, host-only, had no such case).
//  * backend "xgmi" (the in-node switch, xgmi_switch.h) reduces across the
//    ranks of one node; the loopback ("dummy") backend multiplies a rank's
//    own buffer by num_workers instead, so with it init() refuses
//    (ncclInvalidUsage) unless SWITCHML_COLLNET_LOOPBACK=1 says the caller
//    wants exactly that (tests, single-rank benchmarks).
// Configuration: SWITCHML_CONFIG_INI (INI text) or SWITCHML_CONFIG (path),
// else the reference's search path (/etc/switchml.cfg, ./switchml.cfg, ...).
//
// Beside the CollNet table the library exports a p2p net table,
// ncclNetPlugin_v6, as the reference does (switchml_plugin.cc:37): NCCL/RCCL
// take the CollNet table of a library only together with its net table, and
// drop both when that net fails init.  The reference leaves its net table
// empty for a patched NCCL to fill with NCCL's own IB net
// (switchml_nccl.patch:24-81); this library carries its own TCP net
// (socket_net.h), so RCCL keeps the CollNet table with no patch and no other
// plugin.  SWITCHML_NET_PLUGIN=<library exporting ncclNetPlugin_v6> forwards
// the net table to that library instead (e.g. a vendor RDMA net).
//
// switchml_collnet_stats() (C symbol) reports how often RCCL called the
// CollNet entry points, so a run can prove that its all-reduces went through
// iallreduce.
#include <dlfcn.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include <hip/hip_runtime_api.h>

#include "collnet_abi.h"
#include "context.h"
#include "switchml_hip.h"
#include "loopback_backend.h"
#include "job_order.h"
#include "socket_net.h"

namespace {

ncclDebugLogger_t g_logger = nullptr;

// Calls RCCL made into the CollNet table (switchml_collnet_stats()).
struct Counters {
    std::atomic<uint64_t> init{0}, connect{0}, iallreduce{0}, iallreduce_bytes{0}, test_done{0}, reg_mr{0},
        iallreduce_submitted{0}, declined{0};
} g_calls;

void log_info(const char* msg) {
    if (g_logger) g_logger(NCCL_LOG_INFO, ~0ul, __FILE__, __LINE__, "%s", msg);
}

struct ListenComm {
    int dev;
};

struct CollComm {
    int nranks;
    int rank;
    uint32_t ordinal;                    // connect() ordinal in this process
    uint32_t next_mr = 0;                // registration ordinals (job_order.h keys)
    std::map<uint32_t, uint64_t> calls;  // per send-buffer registration: calls so far
};

struct MemHandle {
    int type;
    uint32_t id;
};

struct Request {
    std::shared_ptr<switchml::Job> job;   // null until submitted (job_order.h)
    ncclDataType_t dtype;
    int count;
    void* send;
    void* recv;                           // what the job reduces into
    void* user_recv;                      // caller's recv buffer (uint8 case)
    int32_t* widened;                     // temp int32 buffer (uint8 case, host buffers)
    int32_t* dwidened;                    // temp int32 buffer (uint8 case, device buffers)
    sml_collnet::CallKey key;
    bool failed;
    hipStream_t aux = nullptr;            // aux_stream of dwidened's device (uint8 case, device buffers)
};

// One submission order for every worker of the in-node switch (job_order.h);
// null with the loopback backend or a single worker.  RCCL calls the CollNet
// table from its proxy thread; the mutex makes other callers safe too.
std::mutex g_mu;
std::unique_ptr<sml_collnet::JobOrder> g_order;
std::deque<Request*> g_unsubmitted;   // worker 0: not yet logged (log full); others: waiting for their turn
uint32_t g_comms = 0, g_open_comms = 0;
bool g_trace = false;

int type_size(ncclDataType_t t) {
    switch (t) {
        case ncclUint8: return 1;
        case ncclInt32:
        case ncclFloat32: return 4;
        default: return 0;
    }
}

// Is the caller RCCL?  RCCL hands its own debug logger to init(): the
// library that defines it names the caller.
bool called_by_rccl(ncclDebugLogger_t logger) {
    Dl_info info;
    if (!logger || !dladdr(reinterpret_cast<void*>(logger), &info) || !info.dli_fname) return false;
    return strstr(info.dli_fname, "librccl") != nullptr;
}

ncclResult_t sml_init(ncclDebugLogger_t logger) {
    g_logger = logger;
    g_calls.init++;
    // RCCL 7.2 has no working CollNet all-reduce to hand us (measured on
    // MI355X): its tuner picks CollNetChain, whose kernels
    // it does not build (0 threads), and the AllReduce returns WITHOUT
    // reducing; CollNetDirect needs a switch node in the topology and then
    // never posts the proxy op (the collective hangs).  So under RCCL the
    // CollNet table declines, RCCL logs "Cannot initialize CollNet, using
    // point-to-point network instead" and runs its own algorithms over this
    // library's net.  SWITCHML_COLLNET_RCCL=1 offers the table anyway.
    const char* force = getenv("SWITCHML_COLLNET_RCCL");
    if (called_by_rccl(logger) && !(force && strcmp(force, "1") == 0)) {
        g_calls.declined++;
        if (g_logger)
            g_logger(NCCL_LOG_WARN, ~0ul, __FILE__, __LINE__,
                     "SwitchML CollNet: not offered to RCCL (its CollNet AllReduce paths do not reduce or hang on "
                     "this RCCL; SWITCHML_COLLNET_RCCL=1 overrides)");
        return ncclInvalidUsage;
    }
    try {
        switchml::Context& ctx = switchml::Context::GetInstance();
        if (ctx.GetContextState() == switchml::Context::RUNNING) return ncclSuccess;
        switchml::Config cfg;
        bool have = false;
        if (const char* ini = getenv("SWITCHML_CONFIG_INI")) have = cfg.LoadFromString(ini);
        else if (const char* path = getenv("SWITCHML_CONFIG")) have = cfg.LoadFromFile(path);
        else have = cfg.LoadFromFile();
        if (!have) {
            log_info("SwitchML CollNet: no switchml.cfg found");
            return ncclInvalidUsage;
        }
        // the loopback ("dummy") backend multiplies a rank's own buffer by
        // num_workers instead of summing the ranks' buffers: opt-in only
        const char* lb = getenv("SWITCHML_COLLNET_LOOPBACK");
        if (cfg.general_.backend == "dummy" && (!lb || strcmp(lb, "1") != 0)) {
            if (g_logger)
                g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__,
                         "SwitchML CollNet: the loopback backend does not reduce across ranks; use backend = xgmi, "
                         "or set SWITCHML_COLLNET_LOOPBACK=1 to use it anyway");
            return ncclInvalidUsage;
        }
        return ctx.Start(&cfg) ? ncclSuccess : ncclInternalError;
    } catch (const std::exception& e) {
        if (g_logger) g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__, "SwitchML CollNet init failed: %s", e.what());
        return ncclInternalError;
    }
}

ncclResult_t sml_devices(int* ndev) {
    *ndev = 1;
    return ncclSuccess;
}

char g_name[] = "SWITCHML";

ncclResult_t sml_get_properties(int dev, ncclNetProperties_v6_t* props) {
    if (dev != 0 || !props) return ncclInvalidArgument;
    memset(props, 0, sizeof(*props));
    props->name = g_name;
    props->pciPath = nullptr;    // not a PCI device (the switch is reached through the net)
    props->guid = 0x53574d4cull;  // "SWML"
    props->ptrSupport = NCCL_PTR_HOST | NCCL_PTR_CUDA;
    props->speed = 100000;
    props->port = 0;
    props->latency = 0.0f;
    props->maxComms = 1;         // switchml_plugin.cc:162
    props->maxRecvs = 1;
    return ncclSuccess;
}

ncclResult_t sml_listen(int dev, void* handle, void** listen_comm) {
    if (!handle || !listen_comm) return ncclInvalidArgument;
    memset(handle, 0, NCCL_NET_HANDLE_MAXSIZE);
    memcpy(handle, "SWITCHML", 8);
    *listen_comm = new ListenComm{dev};
    return ncclSuccess;
}

ncclResult_t sml_connect(void* handles[], int nranks, int rank, void* listen_comm, void** coll_comm) {
    (void)handles;
    (void)listen_comm;
    if (rank < 0 || rank >= nranks) return ncclInternalError;  // switchml_plugin.cc:210-213
    // with the in-node switch the communicator must be the session's workers
    const switchml::GeneralConfig& g = switchml::Context::GetInstance().GetConfig().general_;
    if (g.backend == "xgmi" && (nranks != g.num_workers || rank != g.rank)) {
        if (g_logger)
            g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__,
                     "SwitchML CollNet: communicator rank %d of %d, but the xgmi session is worker %d of %d",
                     rank, nranks, (int)g.rank, (int)g.num_workers);
        return ncclInvalidUsage;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (g.backend == "xgmi" && nranks > 1 && !g_order) {
        try {
            const switchml::Config& cfg = switchml::Context::GetInstance().GetConfig();
            g_order.reset(new sml_collnet::JobOrder(cfg.backend_.xgmi.session, rank, nranks,
                                                    cfg.backend_.xgmi.timeout_ms));
        } catch (const std::exception& e) {
            if (g_logger) g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__, "SwitchML CollNet: %s", e.what());
            return ncclSystemError;
        }
    }
    g_trace = getenv("SWITCHML_COLLNET_TRACE") != nullptr;
    g_calls.connect++;
    auto* c = new CollComm;
    c->nranks = nranks;
    c->rank = rank;
    c->ordinal = g_comms++;
    g_open_comms++;
    *coll_comm = c;
    return ncclSuccess;
}

ncclResult_t sml_reduce_support(ncclDataType_t dtype, ncclRedOp_t op, int* supported) {
    *supported = (dtype == ncclFloat32 || dtype == ncclInt32 || dtype == ncclUint8) && op == ncclSum;
    return ncclSuccess;
}

ncclResult_t sml_reg_mr(void* coll_comm, void*, int, int type, void** mhandle) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_calls.reg_mr++;
    auto* c = static_cast<CollComm*>(coll_comm);
    *mhandle = new MemHandle{type, c ? c->next_mr++ : 0u};
    return ncclSuccess;
}

ncclResult_t sml_reg_mr_dmabuf(void* coll_comm, void* data, size_t, int type, uint64_t, int, void** mhandle) {
    return sml_reg_mr(coll_comm, data, 0, type, mhandle);
}

ncclResult_t sml_dereg_mr(void*, void* mhandle) {
    delete static_cast<MemHandle*>(mhandle);
    return ncclSuccess;
}

void submit(Request* r) {
    const switchml::DataType sdt = r->dtype == ncclFloat32 ? switchml::FLOAT32 : switchml::INT32;
    r->job = switchml::Context::GetInstance().AllReduceAsync(r->send, r->recv, (uint64_t)r->count, sdt,
                                                             switchml::SUM);
    g_calls.iallreduce_submitted++;
    if (g_trace && g_logger)
        g_logger(NCCL_LOG_INFO, ~0ul, __FILE__, __LINE__, "SwitchML CollNet: job comm %u buf %u call %lu count %d",
                 r->key.comm, r->key.buf, (unsigned long)r->key.seq, r->count);
}

// Submit whatever the job order allows (job_order.h); g_mu held.
void pump() {
    if (!g_order) return;
    if (g_order->leader()) {
        while (!g_unsubmitted.empty() && g_order->Append(g_unsubmitted.front()->key)) {
            submit(g_unsubmitted.front());
            g_unsubmitted.pop_front();
        }
        return;
    }
    sml_collnet::CallKey k;
    while (g_order->Peek(&k)) {
        auto it = g_unsubmitted.begin();
        for (; it != g_unsubmitted.end(); ++it) {
            const sml_collnet::CallKey& q = (*it)->key;
            if (q.comm == k.comm && q.buf == k.buf && q.seq == k.seq) break;
        }
        if (it == g_unsubmitted.end()) return;   // this rank's call for the entry has not come yet
        Request* r = *it;
        g_unsubmitted.erase(it);
        g_order->Consume();
        if (r->key.count != k.count || r->key.dtype != k.dtype) {
            if (g_logger)
                g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__,
                         "SwitchML CollNet: worker 0 reduces %ld elements of type %d for this call, this worker %ld "
                         "of type %d", (long)k.count, k.dtype, (long)r->key.count, r->key.dtype);
            r->failed = true;
            g_order->Poison();
            continue;
        }
        submit(r);
    }
}

// The plugin's own stream for the uint8 widen / narrow kernels and their
// scratch, one per device: the stream of the device that holds
// the call's buffers, created on that device at its first use, so a process
// that drives several GPUs never runs a kernel or an allocation on another
// device's stream.  Null when the device cannot be determined or the stream
// cannot be created.
hipStream_t aux_stream(int dev) {
    static std::mutex mu;
    static std::map<int, hipStream_t> streams;
    if (dev < 0) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto it = streams.find(dev);
    if (it != streams.end()) return it->second;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || (cur != dev && hipSetDevice(dev) != hipSuccess)) {
        (void)hipGetLastError();
        return nullptr;
    }
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        st = nullptr;
    }
    if (cur != dev) (void)hipSetDevice(cur);
    if (st) streams[dev] = st;
    return st;
}

// The device a device buffer lives on (-1: not a device pointer).
int device_of(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return a.device;
}

// The device scratch is stream-ordered (hipMallocAsync / hipFreeAsync on the
// plugin's stream): hipMalloc / hipFree may synchronise the whole device, and
// RCCL calls iallreduce / test from its proxy thread while its own kernels
// can be waiting on that proxy — a device-wide wait there could deadlock.
void release_widened(Request* r) {
    delete[] r->widened;
    r->widened = nullptr;
    if (r->dwidened) (void)hipFreeAsync(r->dwidened, r->aux);
    r->dwidened = nullptr;
}

ncclResult_t sml_iallreduce(void* coll_comm, void* send, void* recv, int count, ncclDataType_t dtype,
                            ncclRedOp_t op, void* send_mh, void*, void** request) {
    if (op != ncclSum || type_size(dtype) == 0 || count < 0) return ncclInvalidArgument;
    switchml::Context& ctx = switchml::Context::GetInstance();
    if (ctx.GetContextState() != switchml::Context::RUNNING) return ncclInvalidUsage;
    auto* c = static_cast<CollComm*>(coll_comm);
    auto* r = new Request{nullptr, dtype, count, send, recv, recv, nullptr, nullptr, {}, false};
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_order && g_order->Poisoned()) {
        delete r;
        return ncclRemoteError;
    }
    try {
        if (dtype == ncclUint8) {
            const bool ds = switchml::IsDevicePointer(send), dr = switchml::IsDevicePointer(recv);
            if (ds != dr) {                   // one device and one host buffer: not a CollNet call
                delete r;
                return ncclInvalidArgument;
            }
            if (ds) {
                // device buffers: widen on the GPU into a device int32 scratch;
                // the job reads it only after this stream has finished
                hipStream_t st = aux_stream(device_of(send));
                if (device_of(recv) != device_of(send))   // widened scratch and both buffers on one device
                    throw std::runtime_error("uint8 send and recv buffers are on different devices");
                r->aux = st;
                if (!st || hipMallocAsync(reinterpret_cast<void**>(&r->dwidened), 4ull * (count > 0 ? count : 1), st) !=
                               hipSuccess) {
                    (void)hipGetLastError();
                    r->dwidened = nullptr;
                    throw std::runtime_error("allocation of the uint8 widening buffer failed");
                }
                if (sml_widen_u8_i32(static_cast<const uint8_t*>(send), r->dwidened, (uint64_t)count, st) != SML_OK ||
                    hipStreamSynchronize(st) != hipSuccess)
                    throw std::runtime_error("uint8 widening kernel failed");
                r->send = r->recv = r->dwidened;
            } else {
                r->widened = new int32_t[count > 0 ? count : 1];
                const uint8_t* s8 = static_cast<const uint8_t*>(send);
                for (int i = 0; i < count; i++) r->widened[i] = s8[i];
                r->send = r->recv = r->widened;
            }
        }
        const uint32_t buf = send_mh ? static_cast<MemHandle*>(send_mh)->id : 0xffffffffu;
        r->key = {c ? c->ordinal : 0u, buf, c ? c->calls[buf]++ : 0u, (int64_t)count, (int32_t)dtype, 0};
        g_calls.iallreduce++;
        g_calls.iallreduce_bytes += (uint64_t)count * type_size(dtype);
        if (g_order) {
            g_unsubmitted.push_back(r);
            pump();
        } else {
            submit(r);
        }
    } catch (const std::exception& e) {
        if (g_logger) g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__, "SwitchML CollNet: %s", e.what());
        release_widened(r);
        delete r;
        return ncclInternalError;
    }
    *request = r;
    return ncclSuccess;
}

ncclResult_t sml_iflush(void*, void*, int, void*, void** request) {
    // Results are written by the GPU stream of the worker thread and
    // synchronised before the job is marked FINISHED: nothing to flush.
    *request = nullptr;
    return ncclSuccess;
}

ncclResult_t sml_test(void* request, int* done, int* size) {
    Request* r = static_cast<Request*>(request);
    std::lock_guard<std::mutex> lk(g_mu);
    try {
        pump();
    } catch (const std::exception& e) {
        if (g_logger) g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__, "SwitchML CollNet: %s", e.what());
        if (g_order) g_order->Poison();
    }
    const bool poisoned = !r->job && g_order && g_order->Poisoned();
    if (r->failed || poisoned || (r->job && r->job->GetJobStatus() == switchml::FAILED)) {
        *done = 0;
        if (g_order) {
            g_order->Poison();   // the peers' matching jobs cannot complete either
            for (auto it = g_unsubmitted.begin(); it != g_unsubmitted.end(); ++it)
                if (*it == r) {
                    g_unsubmitted.erase(it);
                    break;
                }
        }
        release_widened(r);
        delete r;
        return ncclInternalError;
    }
    if (!r->job || r->job->GetJobStatus() != switchml::FINISHED) {
        *done = 0;
        return ncclSuccess;
    }
    if (r->dtype == ncclUint8) {   // switchml_plugin.cc:370-378
        if (r->dwidened) {
            hipStream_t st = r->aux;   // the stream of the buffers' device (set at widening)
            const bool ok = sml_narrow_i32_u8(r->dwidened, static_cast<uint8_t*>(r->user_recv), (uint64_t)r->count,
                                              st) == SML_OK &&
                            hipStreamSynchronize(st) == hipSuccess;
            release_widened(r);
            if (!ok) {
                delete r;
                return ncclInternalError;
            }
        } else {
            uint8_t* out = static_cast<uint8_t*>(r->user_recv);
            for (int i = 0; i < r->count; i++) out[i] = (uint8_t)r->widened[i];
            release_widened(r);
        }
    }
    *done = 1;
    g_calls.test_done++;
    if (size) *size = r->count * type_size(r->dtype);
    delete r;
    return ncclSuccess;
}

ncclResult_t sml_close_coll(void* coll_comm) {
    std::lock_guard<std::mutex> lk(g_mu);
    delete static_cast<CollComm*>(coll_comm);
    if (g_open_comms && --g_open_comms == 0 && g_unsubmitted.empty()) g_order.reset();
    return ncclSuccess;
}

ncclResult_t sml_close_listen(void* listen_comm) {
    delete static_cast<ListenComm*>(listen_comm);
    return ncclSuccess;
}

// ------------------------------------------------------------ p2p net --
// The built-in TCP net (socket_net.h), or a forwarding table over the net
// plugin named by SWITCHML_NET_PLUGIN.

const ncclNet_v6_t kSocketNet = {
    "SWITCHML",        sml_net::Init,      sml_net::Devices,   sml_net::GetProperties, sml_net::Listen,
    sml_net::Connect,  sml_net::Accept,    sml_net::RegMr,     sml_net::RegMrDmaBuf,   sml_net::DeregMr,
    sml_net::Isend,    sml_net::Irecv,     sml_net::Iflush,    sml_net::Test,          sml_net::CloseSend,
    sml_net::CloseRecv, sml_net::CloseListen};

void* g_net_lib = nullptr;
const ncclNet_v6_t* g_under = nullptr;

ncclResult_t net_init(ncclDebugLogger_t logger) {
    if (logger) g_logger = logger;
    if (g_under) return ncclSuccess;
    const char* path = getenv("SWITCHML_NET_PLUGIN");
    if (!path || !*path) {
        const ncclResult_t r = kSocketNet.init(logger);
        if (r == ncclSuccess) g_under = &kSocketNet;
        return r;
    }
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        if (g_logger) g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__, "SwitchML net: dlopen %s: %s", path, dlerror());
        return ncclInternalError;
    }
    auto* t = static_cast<ncclNet_v6_t*>(dlsym(h, "ncclNetPlugin_v6"));
    if (!t || !t->init) {
        if (g_logger) g_logger(NCCL_LOG_WARN, 0, __FILE__, __LINE__, "SwitchML net: %s has no ncclNetPlugin_v6", path);
        dlclose(h);
        return ncclInternalError;
    }
    const ncclResult_t r = t->init(logger);
    if (r != ncclSuccess) {
        dlclose(h);
        return r;
    }
    g_net_lib = h;
    g_under = t;
    return ncclSuccess;
}

#define SML_FWD(fn, ...)                          \
    do {                                          \
        if (!g_under) return ncclInternalError;   \
        return g_under->fn(__VA_ARGS__);          \
    } while (0)

ncclResult_t net_devices(int* ndev) { SML_FWD(devices, ndev); }
ncclResult_t net_get_properties(int dev, ncclNetProperties_v6_t* props) { SML_FWD(getProperties, dev, props); }
ncclResult_t net_listen(int dev, void* handle, void** listen_comm) { SML_FWD(listen, dev, handle, listen_comm); }
ncclResult_t net_connect(int dev, void* handle, void** send_comm) { SML_FWD(connect, dev, handle, send_comm); }
ncclResult_t net_accept(void* listen_comm, void** recv_comm) { SML_FWD(accept, listen_comm, recv_comm); }
ncclResult_t net_reg_mr(void* comm, void* data, int size, int type, void** mh) {
    SML_FWD(regMr, comm, data, size, type, mh);
}
ncclResult_t net_reg_mr_dmabuf(void* comm, void* data, size_t size, int type, uint64_t off, int fd, void** mh) {
    if (g_under && !g_under->regMrDmaBuf) return ncclInternalError;
    SML_FWD(regMrDmaBuf, comm, data, size, type, off, fd, mh);
}
ncclResult_t net_dereg_mr(void* comm, void* mh) { SML_FWD(deregMr, comm, mh); }
ncclResult_t net_isend(void* send_comm, void* data, int size, int tag, void* mh, void** req) {
    SML_FWD(isend, send_comm, data, size, tag, mh, req);
}
ncclResult_t net_irecv(void* recv_comm, int n, void** data, int* sizes, int* tags, void** mhs, void** req) {
    SML_FWD(irecv, recv_comm, n, data, sizes, tags, mhs, req);
}
ncclResult_t net_iflush(void* recv_comm, int n, void** data, int* sizes, void** mhs, void** req) {
    SML_FWD(iflush, recv_comm, n, data, sizes, mhs, req);
}
ncclResult_t net_test(void* req, int* done, int* sizes) { SML_FWD(test, req, done, sizes); }
ncclResult_t net_close_send(void* c) { SML_FWD(closeSend, c); }
ncclResult_t net_close_recv(void* c) { SML_FWD(closeRecv, c); }
ncclResult_t net_close_listen(void* c) { SML_FWD(closeListen, c); }

#undef SML_FWD

}  // namespace

extern "C" {
// Counts of CollNet calls since the library was loaded: init, connect,
// iallreduce, iallreduce bytes, test() completions, regMr, jobs submitted to
// the Context, inits declined (RCCL).  Returns how many of the n slots it filled.
__attribute__((visibility("default"))) int switchml_collnet_stats(uint64_t* out, int n) {
    const uint64_t v[8] = {g_calls.init.load(),      g_calls.connect.load(),   g_calls.iallreduce.load(),
                           g_calls.iallreduce_bytes.load(), g_calls.test_done.load(), g_calls.reg_mr.load(),
                           g_calls.iallreduce_submitted.load(), g_calls.declined.load()};
    int k = 0;
    for (; k < n && k < 8; k++) out[k] = v[k];
    return k;
}

__attribute__((visibility("default"))) ncclNet_v6_t ncclNetPlugin_v6 = {
    "SWITCHML",         net_init,        net_devices,       net_get_properties, net_listen,
    net_connect,        net_accept,      net_reg_mr,        net_reg_mr_dmabuf,  net_dereg_mr,
    net_isend,          net_irecv,       net_iflush,        net_test,           net_close_send,
    net_close_recv,     net_close_listen};

__attribute__((visibility("default"))) ncclCollNet_v6_t ncclCollNetPlugin_v6 = {
    "SWITCHMLv1",       sml_init,        sml_devices,       sml_get_properties, sml_listen,
    sml_connect,        sml_reduce_support, sml_reg_mr,     sml_reg_mr_dmabuf,  sml_dereg_mr,
    sml_iallreduce,     sml_iflush,      sml_test,          sml_close_coll,     sml_close_listen};
}
