// xgmi_switch.cc — see xgmi_switch.h.
#include "xgmi_switch.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <thread>

#include "switchml_hip.h"

namespace switchml {

namespace {

constexpr uint32_t kMagic = 0x534d4c58u;   // "SMLX"
constexpr int kMaxW = SML_MAX_SWITCH_WORKERS;
constexpr int kMaxT = 16;
constexpr size_t kHandle = sizeof(hipIpcMemHandle_t);

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw SwitchMLFatal(std::string("xgmi switch: ") + what + ": " + hipGetErrorString(e));
}

void sml_ok(int s, const char* what) {
    if (s != SML_OK)
        throw SwitchMLFatal(std::string("xgmi switch: ") + what + ": " + sml_status_string((sml_status_t)s) + " " +
                            sml_last_error());
}

// Reapers of wedged switches (XgmiSwitch::Wedged): how many are still
// waiting for their streams to drain before they free what they hold.
std::mutex g_reap_mu;
std::condition_variable g_reap_cv;
int g_reaping = 0;

}  // namespace

// The session segment (zero-filled when created).
struct alignas(64) ShmBarrier {
    std::atomic<uint32_t> count;
    std::atomic<uint32_t> gen;
    char pad[56];
};

struct ShmPlanes {
    unsigned char exps[kHandle], payload[kHandle], out[kHandle];
    std::atomic<uint32_t> published;
};

struct XgmiShm {
    std::atomic<uint32_t> magic;
    uint32_t W, T, P;
    uint64_t cap;
    std::atomic<int32_t> creator_pid;      // worker 0, which creates the segment (O_EXCL)
    std::atomic<uint32_t> poisoned;        // a worker failed inside an exchange: every later barrier throws
    std::atomic<uint32_t> attached;
    std::atomic<uint32_t> detached;
    uint32_t push;                         // backend.xgmi.push of worker 0 (every worker must match)
    ShmBarrier bar[kMaxT + 1];             // [t]: worker thread t; [kMaxT]: setup / teardown
    ShmPlanes planes[kMaxW][kMaxT];
};

static_assert(std::atomic<uint32_t>::is_always_lock_free, "shared-memory atomics must be lock-free");

namespace {
bool pid_alive(int32_t pid) { return pid > 0 && (kill(pid, 0) == 0 || errno == EPERM); }

// mmap of a segment another process creates: worker 0 sizes it (ftruncate)
// only after its O_EXCL create, so a file opened in between is still 0 bytes
// and touching its mapping would raise SIGBUS.  A segment shorter than
// XgmiShm is "not ready" (or stale): closed, nullptr returned.  Closes fd.
XgmiShm* map_sized(int fd, int prot) {
    struct stat st;
    void* m = MAP_FAILED;
    if (fstat(fd, &st) == 0 && (uint64_t)st.st_size >= sizeof(XgmiShm))
        m = mmap(nullptr, sizeof(XgmiShm), prot, MAP_SHARED, fd, 0);
    close(fd);
    return m == MAP_FAILED ? nullptr : static_cast<XgmiShm*>(m);
}
}  // namespace

// Worker 0 creates the segment (O_EXCL), replacing one left behind by a run
// whose worker 0 is gone; the other workers wait for a segment whose creator
// is alive.  So no worker joins a crashed run's barrier counts or handles.
void XgmiSwitch::OpenSegment() {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    auto fail = [&](const std::string& what) { throw SwitchMLFatal("xgmi switch: " + what); };
    if (rank_ == 0) {
        for (int attempt = 0;; attempt++) {
            const int fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
            if (fd >= 0) {
                created_ = true;
                const bool sized = ftruncate(fd, sizeof(XgmiShm)) == 0;
                void* m = sized ? mmap(nullptr, sizeof(XgmiShm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0)
                                : MAP_FAILED;
                close(fd);
                if (m == MAP_FAILED) fail("mapping " + name_ + ": " + strerror(errno));
                shm_ = static_cast<XgmiShm*>(m);
                shm_->W = (uint32_t)W_;
                shm_->T = (uint32_t)T_;
                shm_->P = P_;
                shm_->cap = cap_;
                shm_->push = push_ ? 1u : 0u;
                shm_->creator_pid.store(getpid());
                shm_->magic.store(kMagic, std::memory_order_release);
                return;
            }
            if (errno != EEXIST || attempt > 3) fail("shm_open " + name_ + ": " + strerror(errno));
            const int fe = shm_open(name_.c_str(), O_RDONLY, 0600);
            if (fe >= 0) {
                // a segment too short to hold the header is stale (its creator
                // died between create and size): replaced below
                if (XgmiShm* o = map_sized(fe, PROT_READ)) {
                    const int32_t pid = o->creator_pid.load();
                    munmap(o, sizeof(XgmiShm));
                    if (pid_alive(pid) && pid != getpid())
                        fail("session " + name_ + " is in use by process " + std::to_string(pid) +
                             " (pick another backend.xgmi.session)");
                }
            }
            fprintf(stderr, "[switchml] xgmi switch: replacing %s left behind by an earlier run\n", name_.c_str());
            shm_unlink(name_.c_str());
        }
    }
    for (;;) {
        const int fd = shm_open(name_.c_str(), O_RDWR, 0600);
        if (fd >= 0) {
            // not yet sized by worker 0: not ready, retry (map_sized)
            if (XgmiShm* s = map_sized(fd, PROT_READ | PROT_WRITE)) {
                void* m = s;
                while (s->magic.load(std::memory_order_acquire) != kMagic &&
                       std::chrono::steady_clock::now() < deadline)
                    std::this_thread::sleep_for(std::chrono::microseconds(200));
                if (s->magic.load(std::memory_order_acquire) == kMagic && pid_alive(s->creator_pid.load())) {
                    shm_ = s;
                    return;
                }
                munmap(m, sizeof(XgmiShm));   // stale: worker 0 replaces it
            }
        }
        if (std::chrono::steady_clock::now() > deadline)
            fail("worker 0 did not open session " + name_ + " within backend.xgmi.timeout_ms");
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
}

XgmiSwitch::XgmiSwitch(const Config& config, int device) {
    const GeneralConfig& g = config.general_;
    rank_ = g.rank;
    W_ = g.num_workers;
    T_ = g.num_worker_threads;
    P_ = (uint32_t)g.packet_numel;
    cap_ = (config.backend_.xgmi.max_slice_numel + 1023) / 1024 * 1024;
    timeout_ms_ = config.backend_.xgmi.timeout_ms;
    round_flags_ = config.backend_.hip.vcl ? SML_FLAG_ROUND_RNE : 0u;
    push_ = config.backend_.xgmi.push;
    fail_setup_ = config.backend_.xgmi.fail_setup;
    if (W_ < 1 || W_ > kMaxW) throw SwitchMLFatal("xgmi switch: num_workers must be 1..16");
    if (T_ < 1 || T_ > kMaxT) throw SwitchMLFatal("xgmi switch: num_worker_threads must be 1..16");
    if (rank_ < 0 || rank_ >= W_) throw SwitchMLFatal("xgmi switch: general.rank must be < num_workers");
    name_ = "/switchml-" + config.backend_.xgmi.session;
    try {
        Setup(device);
    } catch (...) {
        // a worker that joined the session and then failed (e.g. it cannot
        // map a peer's plane: the first contact with another GPU) poisons
        // it, so the peers' first exchange fails at once instead of waiting
        // out backend.xgmi.timeout_ms at a barrier this worker never reaches
        if (attached_) Poison();
        Release();   // no planes, mappings or segment left behind by a failed construction
        throw;
    }
}

void XgmiSwitch::Setup(int device) {
    hip_ok(hipSetDevice(device), "hipSetDevice");
    device_ = device;
    {
        // an earlier switch of this process that wedged still holds peer
        // mappings until its streams drain: wait for its reaper (bounded)
        std::unique_lock<std::mutex> lk(g_reap_mu);
        if (!g_reap_cv.wait_for(lk, std::chrono::milliseconds(timeout_ms_), [] { return g_reaping == 0; }))
            throw SwitchMLFatal("xgmi switch: an earlier session's device work has not finished (its planes and "
                                "peer mappings are still held); restart the process");
    }
    OpenSegment();
    if (shm_->attached.fetch_add(1) >= (uint32_t)W_)
        throw SwitchMLFatal("xgmi switch: session " + name_ + " already has num_workers workers");
    attached_ = true;

    const uint64_t cap_b = (cap_ + 63) / 64 + 64;   // blocks at the smallest packet size, padded
    planes_.resize(T_);
    for (int t = 0; t < T_; t++) {
        ThreadPlanes& tp = planes_[t];
        hip_ok(hipMalloc(&tp.exps, cap_b), "hipMalloc");
        // + W packets of the largest size: the inbox's W rows of ceil(B / W)
        // blocks may exceed B blocks by up to W - 1 (push form)
        hip_ok(hipMalloc(&tp.payload, (cap_ + (uint64_t)kMaxW * 1024) * 4), "hipMalloc");
        hip_ok(hipMalloc(&tp.out, cap_ * 4), "hipMalloc");
        hip_ok(hipMalloc(&tp.gexp, cap_b), "hipMalloc");
        hip_ok(hipStreamCreateWithFlags(&tp.xst, hipStreamNonBlocking), "hipStreamCreate");
        ShmPlanes& sp = shm_->planes[rank_][t];
        hipIpcMemHandle_t h;
        hip_ok(hipIpcGetMemHandle(&h, tp.exps), "hipIpcGetMemHandle");
        memcpy(sp.exps, &h, kHandle);
        hip_ok(hipIpcGetMemHandle(&h, tp.payload), "hipIpcGetMemHandle");
        memcpy(sp.payload, &h, kHandle);
        hip_ok(hipIpcGetMemHandle(&h, tp.out), "hipIpcGetMemHandle");
        memcpy(sp.out, &h, kHandle);
        sp.published.store(1, std::memory_order_release);
    }
    Barrier(kMaxT);   // every worker's handles are published
    // The outcome of this worker's setup is held back until every worker has
    // imported (or failed to import) every peer's planes: a worker that
    // failed must not free its exported planes while a peer is still inside
    // hipIpcOpenMemHandle on them — the importer then hangs in the runtime
    // (measured on MI355X, the N = 8 first-contact rehearsal: > 90 s).
    std::string err;
    if (shm_->W != (uint32_t)W_ || shm_->T != (uint32_t)T_ || shm_->P != P_ || shm_->cap != cap_ ||
        shm_->push != (push_ ? 1u : 0u))
        err = "workers disagree on num_workers / num_worker_threads / packet_numel / max_slice_numel / push";
    else if (fail_setup_)
        err = "injected setup failure (backend.xgmi.fail_setup)";
    else
        try {
            OpenPeers();
        } catch (const std::exception& e) {
            err = e.what();
        }
    Barrier(kMaxT);   // every worker is done importing
    if (!err.empty()) throw SwitchMLFatal(err.rfind("xgmi switch: ", 0) == 0 ? err : "xgmi switch: " + err);
}

// Map every peer's planes of every worker thread (hipIpc; over xGMI on a node).
void XgmiSwitch::OpenPeers() {
    for (int t = 0; t < T_; t++) {
        ThreadPlanes& tp = planes_[t];
        tp.peer_exps.resize(W_);
        tp.peer_payload.resize(W_);
        tp.peer_out.resize(W_);
        for (int w = 0; w < W_; w++) {
            if (w == rank_) {
                tp.peer_exps[w] = tp.exps;
                tp.peer_payload[w] = tp.payload;
                tp.peer_out[w] = tp.out;
                continue;
            }
            const ShmPlanes& sp = shm_->planes[w][t];
            if (!sp.published.load(std::memory_order_acquire)) throw SwitchMLFatal("xgmi switch: peer planes missing");
            void* p;
            hipIpcMemHandle_t h;
            memcpy(&h, sp.exps, kHandle);
            hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
            opened_.push_back(p);
            tp.peer_exps[w] = static_cast<const int8_t*>(p);
            memcpy(&h, sp.payload, kHandle);
            hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
            opened_.push_back(p);
            tp.peer_payload[w] = static_cast<const int32_t*>(p);
            memcpy(&h, sp.out, kHandle);
            hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
            opened_.push_back(p);
            tp.peer_out[w] = static_cast<const float*>(p);
        }
    }
}

// Everything this worker holds, in reverse order of Setup; safe on a
// partially built instance.
void XgmiSwitch::Release() {
    if (Wedged() && (!planes_.empty() || !opened_.empty())) {
        // device work that has not finished may still use the planes, the
        // peer mappings and the streams: a detached reaper frees them once
        // every stream involved has drained (never, if the device is hung)
        fprintf(stderr, "[switchml] xgmi switch: device work did not finish; %zu planes and %zu peer mappings "
                        "are freed once it does\n", planes_.size() * 4, opened_.size());
        struct Remains {
            std::vector<ThreadPlanes> planes;
            std::vector<void*> opened;
            int device;
        };
        auto* rem = new Remains{std::move(planes_), std::move(opened_), device_};
        planes_.clear();
        opened_.clear();
        {
            std::lock_guard<std::mutex> lk(g_reap_mu);
            g_reaping++;
        }
        std::thread([rem] {
            (void)hipSetDevice(rem->device);
            for (ThreadPlanes& tp : rem->planes) {
                if (tp.stuck) (void)hipStreamSynchronize(tp.stuck);
                if (tp.xst) (void)hipStreamSynchronize(tp.xst);
            }
            for (void* p : rem->opened) (void)hipIpcCloseMemHandle(p);
            for (ThreadPlanes& tp : rem->planes) {
                (void)hipFree(tp.exps);
                (void)hipFree(tp.payload);
                (void)hipFree(tp.out);
                (void)hipFree(tp.gexp);
                if (tp.xst) (void)hipStreamDestroy(tp.xst);
            }
            delete rem;
            std::lock_guard<std::mutex> lk(g_reap_mu);
            g_reaping--;
            g_reap_cv.notify_all();
        }).detach();
    }
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    for (ThreadPlanes& tp : planes_) {
        (void)hipFree(tp.exps);
        (void)hipFree(tp.payload);
        (void)hipFree(tp.out);
        (void)hipFree(tp.gexp);
        if (tp.xst) (void)hipStreamDestroy(tp.xst);
    }
    planes_.clear();
    if (!shm_) return;
    bool last = false;
    if (attached_) last = shm_->detached.fetch_add(1) + 1 == (uint32_t)W_;
    const bool poisoned = shm_->poisoned.load() != 0;
    munmap(shm_, sizeof(XgmiShm));
    shm_ = nullptr;
    // the last worker out removes the name; so does worker 0 when the session
    // failed (no peer may join it again)
    if (last || (created_ && poisoned)) shm_unlink(name_.c_str());
}

XgmiSwitch::~XgmiSwitch() {
    if (!shm_) return;
    if (Wedged()) Poison();   // the peers must not wait for this worker's teardown barriers
    if (!shm_->poisoned.load()) {
        try {
            Barrier(kMaxT);   // nobody reads a peer's planes any more
        } catch (...) {
        }
        for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
        opened_.clear();
        try {
            Barrier(kMaxT);   // every mapping of our planes is closed
        } catch (...) {
        }
    }
    Release();
}

void XgmiSwitch::NoteStuckStream(int tid, hipStream_t st) {
    if (tid >= 0 && tid < (int)planes_.size()) planes_[tid].stuck = st;
}

void XgmiSwitch::Poison() {
    if (shm_) shm_->poisoned.store(1, std::memory_order_release);
}

// Sense-reversing barrier over the W workers (one per worker thread, so the
// T slices of a job are exchanged independently).  Polls; a worker that does
// not arrive within backend.xgmi.timeout_ms fails the slice.
void XgmiSwitch::Barrier(int index) {
    ShmBarrier& b = shm_->bar[index];
    if (shm_->poisoned.load(std::memory_order_acquire))
        throw SwitchMLFatal("xgmi switch: the session failed on another worker");
    const uint32_t g = b.gen.load(std::memory_order_acquire);
    if (b.count.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)W_) {
        b.count.store(0, std::memory_order_relaxed);
        b.gen.store(g + 1, std::memory_order_release);
        return;
    }
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    uint32_t spins = 0;
    while (b.gen.load(std::memory_order_acquire) == g) {
        if (++spins > 256) {
            std::this_thread::yield();
            if ((spins & 1023) == 0) {
                // A worker that failed mid-exchange poisons the session: its
                // arrival (or absence) would put every later barrier of this
                // thread index out of phase, so nobody proceeds past it.
                if (shm_->poisoned.load(std::memory_order_acquire))
                    throw SwitchMLFatal("xgmi switch: the session failed on another worker");
                if (std::chrono::steady_clock::now() > deadline) {
                    Poison();
                    throw SwitchMLFatal("xgmi switch: barrier timeout (a worker did not arrive)");
                }
            }
        }
    }
}

bool XgmiSwitch::StreamSync(hipStream_t st, bool bounded_only) {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    for (uint32_t spins = 0;; spins++) {
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) return true;
        if (q != hipErrorNotReady) {
            wedged_.store(true, std::memory_order_release);   // a failed stream: its work's state is unknown
            if (bounded_only) return false;
            hip_ok(q, "hipStreamQuery");
        }
        if (spins > 256) {
            std::this_thread::yield();
            if ((spins & 1023) == 0 && std::chrono::steady_clock::now() > deadline) {
                wedged_.store(true, std::memory_order_release);
                if (bounded_only) return false;
                throw SwitchMLFatal("xgmi switch: device work did not finish within backend.xgmi.timeout_ms");
            }
        }
    }
}

namespace {
// The writer's half of every hand-off to the peers: write
// this GPU's L2 back before the stream sync that precedes the barrier.
void release(hipStream_t st) { sml_ok(sml_release_to_peers(st), "sml_release_to_peers"); }
constexpr uint32_t kPeer = SML_FLAG_PEER_PLANES;   // the reader's half: acquire in the reading kernels
}  // namespace

// The switch's exponent max over the W planes into gexp, then K3: quantize
// with the global exponents into the own BE payload plane (pull), or each
// shard w straight into row `rank` of worker w's inbox (push: one K3 launch
// per shard, W − 1 of them writing over xGMI).
void XgmiSwitch::Quantize(ThreadPlanes& tp, const float* in, uint64_t n, hipStream_t st) {
    const uint64_t B = sml_num_blocks(n, P_);
    sml_ok(sml_switch_exps(tp.peer_exps.data(), (uint16_t)W_, B, tp.gexp, kPeer, st), "sml_switch_exps");
    if (!push_) {
        sml_ok(sml_quantize_pack(in, n, P_, (uint16_t)W_, tp.gexp, tp.payload, nullptr, round_flags_, st),
               "sml_quantize_pack");
        return;
    }
    const uint64_t S = (B + W_ - 1) / W_;
    for (int w = 0; w < W_; w++) {
        const uint64_t b0 = std::min<uint64_t>((uint64_t)w * S, B);
        const uint64_t nb = std::min<uint64_t>(S, B - b0);
        if (!nb) continue;
        const uint64_t n_el = std::min<uint64_t>(nb * P_, n - b0 * P_);
        int32_t* row = const_cast<int32_t*>(tp.peer_payload[w]) + (uint64_t)rank_ * S * P_;
        sml_ok(sml_quantize_pack(in + b0 * P_, n_el, P_, (uint16_t)W_, tp.gexp + b0, row, nullptr, round_flags_, st),
               "sml_quantize_pack");
    }
}

// K6: the wrapping sum of this worker's shard over the W planes, dequantized
// into the own output plane.
void XgmiSwitch::Aggregate(ThreadPlanes& tp, uint64_t n, hipStream_t st) {
    const uint64_t B = sml_num_blocks(n, P_);
    const uint64_t S = (B + W_ - 1) / W_;
    const uint64_t blk0 = std::min<uint64_t>((uint64_t)rank_ * S, B);
    const uint64_t nb = std::min<uint64_t>(S, B - blk0);
    if (!nb) return;
    const uint64_t n_el = std::min<uint64_t>(nb * P_, n - blk0 * P_);
    const int32_t* planes[kMaxW];
    const int8_t* exps[kMaxW];
    for (int w = 0; w < W_; w++) {
        // pull: worker w's plane at this shard; push: row w of the own inbox
        planes[w] = push_ ? tp.payload + (uint64_t)w * S * P_ : tp.peer_payload[w] + blk0 * P_;
        exps[w] = tp.gexp + blk0;
    }
    sml_ok(sml_switch_aggregate(planes, exps, (uint16_t)W_, n_el, P_, nullptr, nullptr, tp.out + blk0 * P_, kPeer,
                                st),
           "sml_switch_aggregate");
}

// A FLOAT32 slice, chunk by chunk, pipelined on two streams (the caller's
// `st` for the local HBM work, tp.xst for the xGMI phases):
//   prologue   K2(0) | barrier | max + K3(0) | barrier
//   chunk c    K6(c) on xst  beside  K2(c+1) on st          | barrier
//              gather(c) on xst  beside  max + K3(c+1) on st | barrier
// Push form: chunk c's phase 1 also writes the own shard into every peer's
// out plane, and phase 2's gather becomes one local copy of the own out plane
// (all W shards are there after the barrier); the out plane is next written
// in chunk c + 1's phase 1, after the barrier that ends phase 2.
// Every plane's readers finish before the barrier that precedes its next
// writer: exps (peers' max of chunk c+1, phase 2) before K2(c+2) (phase 1 of
// the next chunk); payload (peers' K6(c), phase 1) before K3(c+1) (phase 2);
// out (peers' gather(c), phase 2) before K6(c+1); gexp (own K6(c)) before
// the max of chunk c+1.  So one set of planes serves the pipeline.
void XgmiSwitch::FloatSlice(int tid, const float* in, float* out, uint64_t numel, hipStream_t st) {
    ThreadPlanes& tp = planes_[tid];
    const uint64_t nchunks = (numel + cap_ - 1) / cap_;
    auto len = [&](uint64_t c) { return std::min<uint64_t>(cap_, numel - c * cap_); };
    sml_ok(sml_exponents(in, len(0), P_, tp.exps, st), "sml_exponents");
    release(st);
    StreamSync(st);
    Barrier(tid);
    Quantize(tp, in, len(0), st);
    release(st);
    StreamSync(st);
    Barrier(tid);
    for (uint64_t c = 0; c < nchunks; c++) {
        const uint64_t n = len(c), B = sml_num_blocks(n, P_), S = (B + W_ - 1) / W_;
        const bool next = c + 1 < nchunks;
        const float* in_next = in + (c + 1) * cap_;
        Aggregate(tp, n, tp.xst);
        if (push_) PushShard(tp, n, B, S, tp.xst);   // the multicast, as writes into the peers' out planes
        release(tp.xst);
        if (next) {
            sml_ok(sml_exponents(in_next, len(c + 1), P_, tp.exps, st), "sml_exponents");
            release(st);
        }
        StreamSync(tp.xst);
        StreamSync(st);
        Barrier(tid);
        if (push_) {   // every shard is in the own out plane now: one local copy
            const void* src = tp.out;
            void* dst = out + c * cap_;
            sml_ok(sml_copy_segments(&src, &dst, &n, 1, kPeer, tp.xst), "sml_copy_segments");
        } else {
            Gather(tp, out + c * cap_, n, B, S, tp.xst);
        }
        if (next) {
            Quantize(tp, in_next, len(c + 1), st);
            release(st);
        }
        StreamSync(tp.xst);
        StreamSync(st);
        Barrier(tid);   // peers are done reading our planes before they are written again
    }
}

// Push form: this worker's dequantized shard (blocks [rank S, ...) of the own
// out plane) written into the same place of every peer's out plane (W − 1
// segments in one launch, over xGMI), so that after the next barrier every
// out plane holds all W shards.
void XgmiSwitch::PushShard(ThreadPlanes& tp, uint64_t n, uint64_t B, uint64_t S, hipStream_t st) {
    const uint64_t b0 = std::min<uint64_t>((uint64_t)rank_ * S, B);
    const uint64_t nb = std::min<uint64_t>(S, B - b0);
    if (!nb || W_ == 1) return;
    const uint64_t words = std::min<uint64_t>(nb * P_, n - b0 * P_);
    const void* srcs[kMaxW];
    void* dsts[kMaxW];
    uint64_t cnt[kMaxW];
    uint32_t k = 0;
    for (int w = 0; w < W_; w++) {
        if (w == rank_) continue;
        srcs[k] = tp.out + b0 * P_;
        dsts[k] = const_cast<float*>(tp.peer_out[w]) + b0 * P_;
        cnt[k] = words;
        k++;
    }
    sml_ok(sml_copy_segments(srcs, dsts, cnt, k, 0, st), "sml_copy_segments");
}

// Worker w's shard of every plane (blocks [w S, min((w+1) S, B))) from its
// out plane into `out`, one sml_copy_segments launch for the W shards.
void XgmiSwitch::Gather(ThreadPlanes& tp, void* out, uint64_t n, uint64_t B, uint64_t S, hipStream_t st) {
    const void* srcs[kMaxW];
    void* dsts[kMaxW];
    uint64_t words[kMaxW];
    uint32_t k = 0;
    for (int w = 0; w < W_; w++) {
        const uint64_t b0 = std::min<uint64_t>((uint64_t)w * S, B);
        const uint64_t nbw = std::min<uint64_t>(S, B - b0);
        if (!nbw) continue;
        srcs[k] = reinterpret_cast<const uint32_t*>(tp.peer_out[w]) + b0 * P_;
        dsts[k] = static_cast<uint32_t*>(out) + b0 * P_;
        words[k] = std::min<uint64_t>(nbw * P_, n - b0 * P_);
        k++;
    }
    sml_ok(sml_copy_segments(srcs, dsts, words, k, kPeer, st), "sml_copy_segments");
}

void XgmiSwitch::IntChunk(int tid, const int32_t* in, int32_t* out, uint64_t n, hipStream_t st) {
    ThreadPlanes& tp = planes_[tid];
    const uint64_t B = sml_num_blocks(n, P_);
    const uint64_t S = (B + W_ - 1) / W_;
    sml_ok(sml_copy_words(in, tp.payload, n, st), "sml_copy_words");
    release(st);
    StreamSync(st);
    Barrier(tid);
    const uint64_t blk0 = std::min<uint64_t>((uint64_t)rank_ * S, B);
    const uint64_t nb = std::min<uint64_t>(S, B - blk0);
    if (nb) {
        const int32_t* planes[kMaxW];
        for (int w = 0; w < W_; w++) planes[w] = tp.peer_payload[w] + blk0 * P_;
        int32_t* dst = reinterpret_cast<int32_t*>(tp.out) + blk0 * P_;
        sml_ok(sml_switch_aggregate(planes, nullptr, (uint16_t)W_, nb * P_, P_, dst, nullptr, nullptr,
                                    SML_FLAG_PAYLOAD_LE | kPeer, st),
               "sml_switch_aggregate");
        release(st);
    }
    StreamSync(st);
    Barrier(tid);
    Gather(tp, out, n, B, S, st);
    StreamSync(st);
    Barrier(tid);
}

void XgmiSwitch::AllReduceSlice(int tid, const void* in, void* out, uint64_t numel, DataType type, hipStream_t st) {
    if (tid < 0 || tid >= T_) throw SwitchMLFatal("xgmi switch: bad worker thread id");
    if (numel == 0) return;
    if (Wedged()) throw SwitchMLFatal("xgmi switch: an earlier slice's device work did not finish");
    if (shm_->poisoned.load(std::memory_order_acquire))
        throw SwitchMLFatal("xgmi switch: the session failed on another worker");
    try {
        if (type == FLOAT32) {
            FloatSlice(tid, static_cast<const float*>(in), static_cast<float*>(out), numel, st);
            return;
        }
        for (uint64_t off = 0; off < numel; off += cap_) {
            const uint64_t n = std::min<uint64_t>(cap_, numel - off);
            IntChunk(tid, static_cast<const int32_t*>(in) + off, static_cast<int32_t*>(out) + off, n, st);
        }
    } catch (...) {
        // this worker's arrival count is now out of phase with its peers':
        // fail the session for everyone rather than let a barrier pair
        // different phases
        Poison();
        // nothing may still touch the planes when the slice is reported
        // failed — unless a wait already timed out (wedged): then waiting
        // again would only add timeout_ms per stream
        if (!Wedged()) (void)StreamSync(st, true);
        if (!Wedged()) (void)StreamSync(planes_[tid].xst, true);
        throw;
    }
}

}  // namespace switchml
