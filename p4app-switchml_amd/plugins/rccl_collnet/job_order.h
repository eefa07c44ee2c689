// job_order.h — one job order for all workers of a CollNet communicator.
//
// The switch pairs the workers' packets by job and slot, so every worker must
// submit the same all-reduces in the same order (the reference's
// nccl_plugin hands its calls to Context::AllReduceAsync in arrival order,
// switchml_plugin.cc:293-345, and relies on that).  RCCL's proxy thread does
// not guarantee it: it posts the CollNet chunks of its channels as each
// channel's GPU data arrives, so two ranks interleave their channels
// differently (seen on MI355X with 2 CollNet channels: the in-node switch then
// paired chunk k of channel 0 on one rank with a chunk of channel 1 on the
// other).  Within one channel the order is fixed.
//
// So each call gets a key that names it identically on every rank —
// (communicator ordinal, the registration ordinal of its send buffer = the
// channel's buffer, the call's ordinal among that buffer's calls) — and
// worker 0's arrival order becomes everybody's submission order: worker 0
// appends each key to a log in a shared-memory segment as it submits the
// call; worker r submits its calls in log order, holding a call until the
// log reaches it.  No deadlock: a rank's call for log entry i depends only on
// that channel's earlier calls, which precede entry i in worker 0's log too.
#ifndef SWITCHML_AMD_JOB_ORDER_H_
#define SWITCHML_AMD_JOB_ORDER_H_

#include <stdint.h>

#include <string>

namespace sml_collnet {

struct CallKey {
    uint32_t comm;    // connect() ordinal in this process
    uint32_t buf;     // registration ordinal of the send buffer (0xffffffff: unregistered)
    uint64_t seq;     // ordinal of the call among that buffer's calls
    int64_t count;    // checked: every worker's call of one key has the same size / type
    int32_t dtype;
    int32_t pad;
};

struct OrderShm;

class JobOrder {
  public:
    // Opens (worker 0: creates) "/switchml-collnet-<session>" for `nworkers`
    // workers; throws std::runtime_error on failure (stale segment included).
    JobOrder(const std::string& session, int rank, int nworkers, uint64_t timeout_ms);
    ~JobOrder();
    JobOrder(const JobOrder&) = delete;
    JobOrder& operator=(const JobOrder&) = delete;

    bool leader() const { return rank_ == 0; }
    // Worker 0: append `k` (false while the log is full: call again).
    bool Append(const CallKey& k);
    // Workers > 0: the key of the next entry to submit, if worker 0 has logged
    // it; Consume() after submitting it.
    bool Peek(CallKey* k) const;
    void Consume();
    // A failure on any worker poisons the order for all.
    void Poison();
    bool Poisoned() const;

  private:
    std::string name_;
    int rank_, nworkers_;
    OrderShm* shm_ = nullptr;
    uint64_t pos_ = 0;   // worker > 0: next log entry to submit
    uint64_t gen_ = 0;   // the segment's generation (its creator's nonce)
};

}  // namespace sml_collnet

#endif  // SWITCHML_AMD_JOB_ORDER_H_
