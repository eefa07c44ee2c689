// job_order.cc — see job_order.h.
#include "job_order.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace sml_collnet {

namespace {
constexpr uint32_t kMagic = 0x534d4c4fu;   // "SMLO"
constexpr uint64_t kLog = 8192;            // entries in flight (keys not yet consumed by every worker)
constexpr int kMaxWorkers = 16;

bool pid_alive(int32_t pid) { return pid > 0 && (kill(pid, 0) == 0 || errno == EPERM); }
}  // namespace

// mmap of a segment worker 0 creates: it is sized (ftruncate) only after the
// O_EXCL create, so a file opened in between is 0 bytes and touching the
// mapping would raise SIGBUS.  Shorter than OrderShm: not ready (or stale) —
// nullptr.  Closes fd unless keep_fd.
OrderShm* map_sized(int fd, int prot, bool keep_fd = false);

// Remove `name` if it still names the segment open on `fd`, holding an
// exclusive flock on that segment.  Both parties that remove a name — worker
// 0 replacing a segment of its own, and the last worker to close a segment —
// do it through here, so each one's "is the name still that segment?" check
// and its unlink are a single step for the other (the last
// detacher's generation check, then worker 0 replacing the segment, then the
// detacher's unlink would remove the NEW communicator's segment).
void unlink_if_named(const std::string& name, int fd) {
    if (flock(fd, LOCK_EX) != 0) return;
    struct stat a, b;
    const int cur = shm_open(name.c_str(), O_RDONLY, 0600);
    const bool same = cur >= 0 && fstat(fd, &a) == 0 && fstat(cur, &b) == 0 && a.st_ino == b.st_ino &&
                      a.st_dev == b.st_dev;
    if (cur >= 0) close(cur);
    if (same) shm_unlink(name.c_str());
    flock(fd, LOCK_UN);
}

struct alignas(64) Counter {
    std::atomic<uint64_t> v;
    char pad[56];
};

struct OrderShm {
    std::atomic<uint32_t> magic;
    uint32_t nworkers;
    std::atomic<int32_t> creator_pid;
    std::atomic<uint32_t> poisoned;
    std::atomic<uint32_t> attached;
    std::atomic<uint32_t> detached;
    uint64_t generation;           // set by the creator: which segment of this name it is
    Counter head;                  // entries worker 0 appended
    Counter done[kMaxWorkers];     // entries each worker > 0 consumed
    CallKey log[kLog];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory atomics must be lock-free");

OrderShm* map_sized(int fd, int prot, bool keep_fd) {
    struct stat st;
    void* m = MAP_FAILED;
    if (fstat(fd, &st) == 0 && (uint64_t)st.st_size >= sizeof(OrderShm))
        m = mmap(nullptr, sizeof(OrderShm), prot, MAP_SHARED, fd, 0);
    if (!keep_fd) close(fd);
    return m == MAP_FAILED ? nullptr : static_cast<OrderShm*>(m);
}

JobOrder::JobOrder(const std::string& session, int rank, int nworkers, uint64_t timeout_ms)
    : name_("/switchml-collnet-" + session), rank_(rank), nworkers_(nworkers) {
    if (nworkers < 1 || nworkers > kMaxWorkers || rank < 0 || rank >= nworkers)
        throw std::runtime_error("job order: bad rank / worker count");
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    auto expired = [&] { return std::chrono::steady_clock::now() > deadline; };
    void* m = MAP_FAILED;
    if (rank == 0) {
        for (int attempt = 0;; attempt++) {
            const int fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
            if (fd >= 0) {
                if (ftruncate(fd, sizeof(OrderShm)) != 0) {
                    close(fd);
                    shm_unlink(name_.c_str());
                    throw std::runtime_error("job order: ftruncate " + name_ + ": " + strerror(errno));
                }
                m = mmap(nullptr, sizeof(OrderShm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
                close(fd);
                if (m == MAP_FAILED) {
                    shm_unlink(name_.c_str());
                    throw std::runtime_error("job order: mmap: " + std::string(strerror(errno)));
                }
                break;
            }
            if (errno != EEXIST || attempt > 3)
                throw std::runtime_error("job order: shm_open " + name_ + ": " + strerror(errno));
            // a segment of that name exists: live (another job uses the session
            // name) or left by a crashed run (its creator is gone): replace it
            // (a segment too short for the header is stale: its creator died
            // between create and size; one created by this process is an
            // earlier communicator's that was never closed)
            const int fe = shm_open(name_.c_str(), O_RDWR, 0600);
            if (fe >= 0) {
                if (OrderShm* o = map_sized(fe, PROT_READ, true)) {
                    const int32_t pid = o->creator_pid.load();
                    munmap(o, sizeof(OrderShm));
                    if (pid_alive(pid) && pid != getpid()) {
                        close(fe);
                        throw std::runtime_error("job order: session " + name_ + " is in use by process " +
                                                 std::to_string(pid));
                    }
                }
                unlink_if_named(name_, fe);
                close(fe);
            }
        }
        shm_ = static_cast<OrderShm*>(m);
        shm_->generation = gen_ = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^
                                  ((uint64_t)getpid() << 40);
        shm_->nworkers = (uint32_t)nworkers;
        shm_->creator_pid.store(getpid());
        shm_->attached.store(1);
        shm_->magic.store(kMagic, std::memory_order_release);
        return;
    }
    // workers > 0: wait for worker 0's live segment
    for (;;) {
        const int fd = shm_open(name_.c_str(), O_RDWR, 0600);
        if (fd >= 0) {
            if (OrderShm* s = map_sized(fd, PROT_READ | PROT_WRITE)) {
                m = s;
                while (s->magic.load(std::memory_order_acquire) != kMagic && !expired())
                    std::this_thread::sleep_for(std::chrono::microseconds(200));
                if (s->magic.load(std::memory_order_acquire) == kMagic && pid_alive(s->creator_pid.load())) {
                    if (s->nworkers != (uint32_t)nworkers) {
                        munmap(m, sizeof(OrderShm));
                        throw std::runtime_error("job order: workers disagree on the worker count");
                    }
                    // One segment serves one communicator: nworkers
                    // attachments (worker 0's included).  A full one is an
                    // earlier communicator's, still open on worker 0 (this
                    // worker closed and reconnected first): its log is not
                    // ours — wait for worker 0's new segment.
                    uint32_t a = s->attached.load();
                    while (a < (uint32_t)nworkers && !s->attached.compare_exchange_weak(a, a + 1)) {
                    }
                    if (a < (uint32_t)nworkers) {
                        shm_ = s;
                        gen_ = s->generation;
                        return;
                    }
                }
                munmap(m, sizeof(OrderShm));   // stale (creator gone) or full: wait for worker 0's
            }
        }
        if (expired()) throw std::runtime_error("job order: worker 0 did not create " + name_ + " in time");
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
}

// The last worker to close removes the name — if the name still is ITS
// segment: worker 0 may already have replaced it with a reconnected
// communicator's (a new generation), which stays.  The generation says the
// fd is this communicator's segment; unlink_if_named makes "the name still
// refers to it" and the unlink one step against worker 0's replacement.
JobOrder::~JobOrder() {
    if (!shm_) return;
    const bool last = shm_->detached.fetch_add(1) + 1 == (uint32_t)nworkers_;
    munmap(shm_, sizeof(OrderShm));
    if (!last) return;
    const int fd = shm_open(name_.c_str(), O_RDONLY, 0600);
    if (fd < 0) return;
    if (OrderShm* s = map_sized(fd, PROT_READ, true)) {
        const bool mine = s->generation == gen_;
        munmap(s, sizeof(OrderShm));
        if (mine) unlink_if_named(name_, fd);   // still this segment under the lock worker 0 replaces with
    }
    close(fd);
}

bool JobOrder::Append(const CallKey& k) {
    const uint64_t h = shm_->head.v.load(std::memory_order_relaxed);
    for (int r = 1; r < nworkers_; r++)
        if (h - shm_->done[r].v.load(std::memory_order_acquire) >= kLog) return false;
    shm_->log[h % kLog] = k;
    shm_->head.v.store(h + 1, std::memory_order_release);
    return true;
}

bool JobOrder::Peek(CallKey* k) const {
    if (pos_ >= shm_->head.v.load(std::memory_order_acquire)) return false;
    *k = shm_->log[pos_ % kLog];
    return true;
}

void JobOrder::Consume() {
    pos_++;
    shm_->done[rank_].v.store(pos_, std::memory_order_release);
}

void JobOrder::Poison() { shm_->poisoned.store(1, std::memory_order_release); }

bool JobOrder::Poisoned() const { return shm_->poisoned.load(std::memory_order_acquire) != 0; }

}  // namespace sml_collnet
