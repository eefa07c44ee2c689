// socket_net.cc — see socket_net.h.
#include "socket_net.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <net/if.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <random>

namespace sml_net {

namespace {

constexpr uint64_t kMagic = 0x534d4c4e45543031ull;   // "SMLNET01"
constexpr int kMaxRequests = 64;                     // per comm; NCCL posts at most NCCL_NET_MAX_REQUESTS

ncclDebugLogger_t g_log = nullptr;
in_addr g_addr{};
char g_ifname[IF_NAMESIZE + 1] = "lo";
char g_name[] = "SWITCHML";   // same name as the CollNet device: RCCL's topology pairs them by name

#define SML_WARN(...) \
    do { if (g_log) g_log(NCCL_LOG_WARN, ~0ul, __FILE__, __LINE__, __VA_ARGS__); } while (0)
#define SML_INFO(...) \
    do { if (g_log) g_log(NCCL_LOG_INFO, ~0ul, __FILE__, __LINE__, __VA_ARGS__); } while (0)

struct WireHandle {   // inside RCCL's 128-byte handle
    uint64_t magic;
    uint32_t ip;      // network order
    uint16_t port;    // network order
    uint16_t pad;
    uint64_t nonce;   // the connector proves it read this handle
};
static_assert(sizeof(WireHandle) <= NCCL_NET_HANDLE_MAXSIZE, "handle too large");

struct MsgHeader {
    uint32_t size;
    uint32_t tag;
};

struct Comm;

struct Request {
    Comm* comm = nullptr;
    bool used = false;
    bool done = false;
    char* data = nullptr;
    uint32_t size = 0;     // send: bytes to send; recv: capacity
    uint32_t got = 0;      // recv: the sender's size
    MsgHeader hdr{};
    uint32_t hdr_off = 0;
    uint64_t off = 0;
};

struct Comm {
    int fd = -1;
    bool is_send = false;
    ncclResult_t error = ncclSuccess;   // sticky: the connection is unusable after it
    Request req[kMaxRequests];
    Request* queue[kMaxRequests];   // posted, in order
    uint32_t head = 0, tail = 0;    // queue indices, mod kMaxRequests
};

struct ListenComm {
    int fd = -1;
    uint64_t nonce = 0;
    int pending = -1;               // accepted, nonce not read yet
    uint64_t got_nonce = 0;
    uint32_t got = 0;
};

bool set_nonblocking(int fd) {
    const int fl = fcntl(fd, F_GETFL, 0);
    return fl >= 0 && fcntl(fd, F_SETFL, fl | O_NONBLOCK) == 0;
}

void set_nodelay(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

uint64_t fresh_nonce() {
    static std::atomic<uint64_t> ctr{0};
    std::random_device rd;
    return ((uint64_t)rd() << 32 ^ (uint64_t)rd()) + ctr.fetch_add(1);
}

// Pick the address peers connect to (socket_net.h).
void choose_address() {
    if (const char* a = getenv("SWITCHML_NET_IFADDR")) {
        if (inet_pton(AF_INET, a, &g_addr) == 1) {
            strcpy(g_ifname, "env");
            return;
        }
        SML_WARN("NET/SWITCHML : SWITCHML_NET_IFADDR=%s is not an IPv4 address, ignored", a);
    }
    const char* prefix = getenv("SWITCHML_NET_IFNAME");
    g_addr.s_addr = htonl(INADDR_LOOPBACK);
    strcpy(g_ifname, "lo");
    ifaddrs* ifs = nullptr;
    if (getifaddrs(&ifs) != 0) return;
    for (ifaddrs* i = ifs; i; i = i->ifa_next) {
        if (!i->ifa_addr || i->ifa_addr->sa_family != AF_INET) continue;
        if (!(i->ifa_flags & IFF_UP) || (i->ifa_flags & IFF_LOOPBACK)) continue;
        if (prefix && *prefix && strncmp(i->ifa_name, prefix, strlen(prefix)) != 0) continue;
        g_addr = reinterpret_cast<sockaddr_in*>(i->ifa_addr)->sin_addr;
        strncpy(g_ifname, i->ifa_name, IF_NAMESIZE);
        g_ifname[IF_NAMESIZE] = 0;
        break;
    }
    freeifaddrs(ifs);
}

// Move the head request(s) of `c` forward as far as the socket allows.
ncclResult_t progress(Comm* c) {
    if (c->error != ncclSuccess) return c->error;
    while (c->head != c->tail) {
        Request* r = c->queue[c->head % kMaxRequests];
        if (c->is_send) {
            while (r->hdr_off < sizeof(MsgHeader) || r->off < r->size) {
                iovec iov[2];
                int n = 0;
                if (r->hdr_off < sizeof(MsgHeader))
                    iov[n++] = {reinterpret_cast<char*>(&r->hdr) + r->hdr_off, sizeof(MsgHeader) - r->hdr_off};
                if (r->off < r->size) iov[n++] = {r->data + r->off, r->size - r->off};
                msghdr m{};
                m.msg_iov = iov;
                m.msg_iovlen = n;
                const ssize_t s = sendmsg(c->fd, &m, MSG_NOSIGNAL | MSG_DONTWAIT);
                if (s < 0) {
                    if (errno == EAGAIN || errno == EWOULDBLOCK) return ncclSuccess;
                    if (errno == EINTR) continue;
                    SML_WARN("NET/SWITCHML : send failed: %s", strerror(errno));
                    return c->error = ncclRemoteError;
                }
                uint64_t k = (uint64_t)s;
                const uint32_t h = std::min<uint64_t>(k, sizeof(MsgHeader) - r->hdr_off);
                r->hdr_off += h;
                r->off += k - h;
            }
        } else {
            while (r->hdr_off < sizeof(MsgHeader)) {
                const ssize_t s = recv(c->fd, reinterpret_cast<char*>(&r->hdr) + r->hdr_off,
                                       sizeof(MsgHeader) - r->hdr_off, MSG_DONTWAIT);
                if (s < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return ncclSuccess;
                if (s < 0 && errno == EINTR) continue;
                if (s <= 0) {
                    SML_WARN("NET/SWITCHML : connection closed by peer (%s)", s < 0 ? strerror(errno) : "EOF");
                    return c->error = ncclRemoteError;
                }
                r->hdr_off += (uint32_t)s;
                if (r->hdr_off == sizeof(MsgHeader)) {
                    if (r->hdr.size > r->size) {
                        SML_WARN("NET/SWITCHML : message of %u bytes for a %u-byte receive", r->hdr.size, r->size);
                        return c->error = ncclInternalError;
                    }
                    r->got = r->hdr.size;
                }
            }
            while (r->off < r->got) {
                const ssize_t s = recv(c->fd, r->data + r->off, r->got - r->off, MSG_DONTWAIT);
                if (s < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return ncclSuccess;
                if (s < 0 && errno == EINTR) continue;
                if (s <= 0) {
                    SML_WARN("NET/SWITCHML : connection closed by peer (%s)", s < 0 ? strerror(errno) : "EOF");
                    return c->error = ncclRemoteError;
                }
                r->off += (uint64_t)s;
            }
        }
        r->done = true;
        c->head++;
    }
    return ncclSuccess;
}

Request* post(Comm* c, void* data, uint32_t size, uint32_t tag) {
    if (c->tail - c->head >= (uint32_t)kMaxRequests) return nullptr;
    for (Request& r : c->req) {
        if (r.used) continue;
        r = Request{};
        r.comm = c;
        r.used = true;
        r.data = static_cast<char*>(data);
        r.size = size;
        r.hdr = {size, (uint32_t)tag};
        c->queue[c->tail++ % kMaxRequests] = &r;
        return &r;
    }
    return nullptr;
}

}  // namespace

ncclResult_t Init(ncclDebugLogger_t logger) {
    g_log = logger;
    choose_address();
    char ip[INET_ADDRSTRLEN] = "?";
    inet_ntop(AF_INET, &g_addr, ip, sizeof(ip));
    SML_INFO("NET/SWITCHML : TCP net on %s (%s)", g_ifname, ip);
    return ncclSuccess;
}

ncclResult_t Devices(int* ndev) {
    *ndev = 1;
    return ncclSuccess;
}

ncclResult_t GetProperties(int dev, ncclNetProperties_v6_t* props) {
    if (dev != 0 || !props) return ncclInvalidArgument;
    memset(props, 0, sizeof(*props));
    props->name = g_name;
    props->pciPath = nullptr;           // not a PCI device: RCCL attaches it to the CPU
    props->guid = 0x53574d4cull;        // the CollNet device's guid ("SWML")
    props->ptrSupport = NCCL_PTR_HOST;
    props->speed = 100000;
    props->port = 0;
    props->latency = 0.0f;
    props->maxComms = 65536;
    props->maxRecvs = 1;
    return ncclSuccess;
}

ncclResult_t Listen(int dev, void* handle, void** listen_comm) {
    if (dev != 0 || !handle || !listen_comm) return ncclInvalidArgument;
    const int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return ncclSystemError;
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    a.sin_port = 0;
    socklen_t len = sizeof(a);
    if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(fd, 128) != 0 ||
        getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len) != 0 || !set_nonblocking(fd)) {
        SML_WARN("NET/SWITCHML : listen failed: %s", strerror(errno));
        close(fd);
        return ncclSystemError;
    }
    auto* l = new ListenComm;
    l->fd = fd;
    l->nonce = fresh_nonce();
    memset(handle, 0, NCCL_NET_HANDLE_MAXSIZE);
    WireHandle h{kMagic, g_addr.s_addr, a.sin_port, 0, l->nonce};
    memcpy(handle, &h, sizeof(h));
    *listen_comm = l;
    return ncclSuccess;
}

ncclResult_t Connect(int dev, void* handle, void** send_comm) {
    if (dev != 0 || !handle || !send_comm) return ncclInvalidArgument;
    WireHandle h;
    memcpy(&h, handle, sizeof(h));
    if (h.magic != kMagic) {
        SML_WARN("NET/SWITCHML : connect: not a SwitchML net handle");
        return ncclInvalidArgument;
    }
    const int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return ncclSystemError;
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = h.ip;
    a.sin_port = h.port;
    // the peer's socket is listening already (RCCL sends the handle after
    // listen), so the connection completes in its backlog
    int rc;
    do {
        rc = connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a));
    } while (rc != 0 && errno == EINTR);
    if (rc != 0) {
        SML_WARN("NET/SWITCHML : connect failed: %s", strerror(errno));
        close(fd);
        return ncclRemoteError;
    }
    const char* p = reinterpret_cast<const char*>(&h.nonce);
    for (size_t off = 0; off < sizeof(h.nonce);) {
        const ssize_t s = send(fd, p + off, sizeof(h.nonce) - off, MSG_NOSIGNAL);
        if (s < 0 && errno == EINTR) continue;
        if (s <= 0) {
            close(fd);
            return ncclRemoteError;
        }
        off += (size_t)s;
    }
    set_nodelay(fd);
    if (!set_nonblocking(fd)) {
        close(fd);
        return ncclSystemError;
    }
    auto* c = new Comm;
    c->fd = fd;
    c->is_send = true;
    *send_comm = c;
    return ncclSuccess;
}

ncclResult_t Accept(void* listen_comm, void** recv_comm) {
    auto* l = static_cast<ListenComm*>(listen_comm);
    if (!l || !recv_comm) return ncclInvalidArgument;
    *recv_comm = nullptr;
    if (l->pending < 0) {
        const int fd = accept4(l->fd, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK);
        if (fd < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) return ncclSuccess;   // call again
            SML_WARN("NET/SWITCHML : accept failed: %s", strerror(errno));
            return ncclSystemError;
        }
        l->pending = fd;
        l->got = 0;
    }
    char* p = reinterpret_cast<char*>(&l->got_nonce);
    while (l->got < sizeof(l->got_nonce)) {
        const ssize_t s = recv(l->pending, p + l->got, sizeof(l->got_nonce) - l->got, MSG_DONTWAIT);
        if (s < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) return ncclSuccess;
        if (s <= 0) {
            close(l->pending);
            l->pending = -1;
            return ncclSuccess;   // a connector that went away: wait for the next
        }
        l->got += (uint32_t)s;
    }
    const int fd = l->pending;
    l->pending = -1;
    if (l->got_nonce != l->nonce) {   // not the peer this handle was given to
        SML_WARN("NET/SWITCHML : accept: connection with a foreign handle dropped");
        close(fd);
        return ncclSuccess;
    }
    set_nodelay(fd);
    auto* c = new Comm;
    c->fd = fd;
    c->is_send = false;
    *recv_comm = c;
    return ncclSuccess;
}

ncclResult_t RegMr(void*, void*, int, int type, void** mhandle) {
    if (type != NCCL_PTR_HOST) return ncclInternalError;
    *mhandle = nullptr;
    return ncclSuccess;
}

ncclResult_t RegMrDmaBuf(void*, void*, size_t, int, uint64_t, int, void**) { return ncclInternalError; }

ncclResult_t DeregMr(void*, void*) { return ncclSuccess; }

ncclResult_t Isend(void* send_comm, void* data, int size, int tag, void*, void** request) {
    auto* c = static_cast<Comm*>(send_comm);
    if (!c || !c->is_send || size < 0 || !request) return ncclInvalidArgument;
    Request* r = post(c, data, (uint32_t)size, (uint32_t)tag);
    *request = r;   // NULL: no request slot free, RCCL posts again
    return r ? progress(c) : ncclSuccess;
}

ncclResult_t Irecv(void* recv_comm, int n, void** data, int* sizes, int* tags, void**, void** request) {
    auto* c = static_cast<Comm*>(recv_comm);
    if (!c || c->is_send || !request) return ncclInvalidArgument;
    if (n != 1) return ncclInternalError;   // maxRecvs = 1
    if (sizes[0] < 0) return ncclInvalidArgument;
    Request* r = post(c, data[0], (uint32_t)sizes[0], tags ? (uint32_t)tags[0] : 0);
    *request = r;
    return r ? progress(c) : ncclSuccess;
}

ncclResult_t Iflush(void*, int, void**, int*, void**, void** request) {
    *request = nullptr;   // host memory: nothing to flush
    return ncclSuccess;
}

ncclResult_t Test(void* request, int* done, int* sizes) {
    auto* r = static_cast<Request*>(request);
    if (!r || !r->used || !done) return ncclInvalidArgument;
    const ncclResult_t st = progress(r->comm);
    if (st != ncclSuccess) return st;
    *done = r->done ? 1 : 0;
    if (r->done) {
        if (sizes) sizes[0] = (int)(r->comm->is_send ? r->size : r->got);
        r->used = false;
    }
    return ncclSuccess;
}

ncclResult_t CloseSend(void* send_comm) {
    auto* c = static_cast<Comm*>(send_comm);
    if (c) {
        close(c->fd);
        delete c;
    }
    return ncclSuccess;
}

ncclResult_t CloseRecv(void* recv_comm) { return CloseSend(recv_comm); }

ncclResult_t CloseListen(void* listen_comm) {
    auto* l = static_cast<ListenComm*>(listen_comm);
    if (l) {
        if (l->pending >= 0) close(l->pending);
        close(l->fd);
        delete l;
    }
    return ncclSuccess;
}

}  // namespace sml_net
