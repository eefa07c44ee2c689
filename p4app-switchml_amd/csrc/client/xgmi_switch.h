// xgmi_switch.h — the in-node switch backend (general.backend = "xgmi").
//
// The reference's workers send every packet to a Tofino switch, which adds
// the W workers' payload slots as wrapping bit<32> (p4/processor.p4:48-54),
// takes the signed int8 max of their exponents (p4/exponents.p4:48-54) and
// multicasts the result (the DPDK / RDMA backends, out of scope here).  On
// one MI355X node the W workers are W processes, one GPU each, connected by
// xGMI; this backend is their switch without a switch:
//
//   * rendezvous: a POSIX shared-memory segment named by
//     backend.xgmi.session (the role of the controller's gRPC session setup,
//     switchml.proto:21-91) holds every worker thread's plane IPC handles and
//     one barrier per worker thread.  Worker 0 creates it (O_EXCL; a segment
//     left by a crashed run whose worker 0 is gone is replaced), the others
//     wait for it; a worker failing inside an exchange poisons the session so
//     every peer's slices fail instead of pairing out-of-phase barriers;
//   * per FIFO slice (thread t of every worker, the same slice geometry on all
//     workers, as the switch's slots are), chunk by chunk: K2 exponents into
//     the own plane → barrier → the max over the W exponent planes
//     (sml_switch_exps) → K3 quantize with the global exponents into the own
//     BE payload plane → barrier → K6 on this worker's shard of ceil(B / W)
//     blocks, reading the W payload planes (W − 1 over xGMI) and writing the
//     dequantized fp32 shard into the own output plane → barrier → every
//     worker gathers the W shards into its tensor (the multicast, one
//     sml_copy_segments launch) → barrier.  FLOAT32 slices of several chunks
//     are pipelined on two streams: chunk c's K6 runs beside chunk c + 1's K2
//     and chunk c's gather beside chunk c + 1's exponent max and K3 (local
//     HBM work beside the xGMI phases), two barriers per chunk; one set of
//     planes suffices because every plane's readers finish one phase before
//     its next writer starts (xgmi_switch.cc, FloatSlice);
//   * push form (backend.xgmi.push): K3 writes each shard of the quantized
//     payload straight into its owner's inbox plane (W − 1 shards over xGMI,
//     posted writes) and K6 reads the W rows of the own inbox from local HBM;
//     the multicast likewise writes the own dequantized shard into every
//     peer's out plane, and the gather becomes one local copy; same phases,
//     barriers and bytes, every xGMI transfer a write;
//   * INT32 slices: the words themselves are summed (the INT32 PPP only
//     reorders bytes, ppp.cc:158-190, 262-298), pulled in both forms.
// Results are bit-identical to the oracle's W-worker software switch
// (orc_switch_exps / orc_switch_payload + dequantize), slice by slice.
//
// All workers must submit the same jobs (same sizes, same order) — the
// contract the real switch imposes too.  Slices larger than
// backend.xgmi.max_slice_numel are exchanged in chunks of that many elements
// (a multiple of every packet size, so block boundaries do not move).
#ifndef SWITCHML_AMD_XGMI_SWITCH_H_
#define SWITCHML_AMD_XGMI_SWITCH_H_

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <string>
#include <vector>

#include "common.h"
#include "config.h"

namespace switchml {

struct XgmiShm;

class XgmiSwitch {
  public:
    // Opens / creates the session segment, allocates this worker's planes for
    // every worker thread, publishes their IPC handles and maps the peers'
    // (a barrier over all W workers).  Throws SwitchMLFatal on failure.
    XgmiSwitch(const Config& config, int device);
    // Barrier with the other workers, unmap the peers' planes, barrier, free;
    // the last worker removes the segment.  (A poisoned session skips the
    // barriers.)
    ~XgmiSwitch();
    XgmiSwitch(const XgmiSwitch&) = delete;
    XgmiSwitch& operator=(const XgmiSwitch&) = delete;

    // All-reduce worker thread `tid`'s slice across the W workers.  in / out
    // are device-accessible (HBM or pinned host), may alias; returns when the
    // result is in `out` (the stream is synchronised).
    void AllReduceSlice(int tid, const void* in, void* out, uint64_t numel, DataType type, hipStream_t stream);

    // Fail the session for every worker: their next (or current) barrier
    // throws, so their slices fail instead of pairing out-of-phase barriers.
    // AllReduceSlice does this itself when it throws; the fault injection
    // (backend.dummy.fail_worker_thread) calls it too.
    void Poison();

    // Wait for the work queued on a worker's stream for at most
    // backend.xgmi.timeout_ms; never throws.  False: the device did not
    // finish (or failed) — the switch is then wedged.
    bool WaitBounded(hipStream_t st) { return StreamSync(st, true); }
    // A wait on this worker's device work timed out: kernels of this switch
    // may still be reading or writing its planes (or a peer's, over xGMI),
    // and they may never finish.  Nothing on the worker threads waits on
    // that device work again: the failing slices return at once, and
    // teardown hands the planes, peer mappings and streams to a detached
    // reaper thread that frees them only once the stuck streams have
    // drained (hipFree / hipStreamDestroy / hipIpcCloseMemHandle under
    // running kernels would block, or pull memory from under them).  A new
    // switch in the same process first waits (bounded) for earlier reapers:
    // a peer mapping still open from a wedged session could otherwise alias
    // a peer's new plane.
    bool Wedged() const { return wedged_.load(std::memory_order_acquire); }
    // Worker thread `tid`'s stream `st` (the caller's, not the switch's) was
    // abandoned with work still queued: the reaper waits for it too.  The
    // caller keeps the stream alive (never destroys it).
    void NoteStuckStream(int tid, hipStream_t st);

  private:
    struct ThreadPlanes {
        int8_t* exps = nullptr;        // own planes (IPC-exported)
        // the own BE payload plane (pull), or this worker's inbox (push): W
        // rows of S blocks, row r = worker r's quantized share of this
        // worker's shard
        int32_t* payload = nullptr;
        float* out = nullptr;
        int8_t* gexp = nullptr;        // local: the global exponents
        std::vector<const int8_t*> peer_exps;      // [W], own included
        std::vector<const int32_t*> peer_payload;  // [W]
        std::vector<const float*> peer_out;        // [W]
        hipStream_t xst = nullptr;     // the exchange stream (K6, gather) beside the caller's
        hipStream_t stuck = nullptr;   // the caller's stream, abandoned with work queued (NoteStuckStream)
    };

    void OpenSegment();
    void Setup(int device);
    void OpenPeers();
    void Release();
    void Barrier(int index);
    // Wait for the work queued on `st`, polling against backend.xgmi.timeout_ms
    // (a device that never finishes fails the slice instead of blocking the
    // worker thread forever); `bounded_only` waits never throw (cleanup paths).
    bool StreamSync(hipStream_t st, bool bounded_only = false);
    void FloatSlice(int tid, const float* in, float* out, uint64_t numel, hipStream_t st);
    void Aggregate(ThreadPlanes& tp, uint64_t n, hipStream_t st);
    void Quantize(ThreadPlanes& tp, const float* in, uint64_t n, hipStream_t st);
    void IntChunk(int tid, const int32_t* in, int32_t* out, uint64_t n, hipStream_t st);
    void Gather(ThreadPlanes& tp, void* out, uint64_t n, uint64_t B, uint64_t S, hipStream_t st);
    void PushShard(ThreadPlanes& tp, uint64_t n, uint64_t B, uint64_t S, hipStream_t st);

    int rank_, W_, T_;
    int device_ = -1;
    uint32_t P_;
    uint64_t cap_;          // elements per chunk (multiple of 1024)
    uint64_t timeout_ms_;
    uint32_t round_flags_ = 0;   // SML_FLAG_ROUND_RNE under backend.hip.vcl
    bool push_ = false;     // backend.xgmi.push: K3 writes into the owners' inboxes
    bool fail_setup_ = false;   // backend.xgmi.fail_setup (fault injection)
    std::string name_;
    XgmiShm* shm_ = nullptr;
    bool created_ = false;    // this worker (rank 0) created the segment
    bool attached_ = false;   // counted in shm_->attached
    std::vector<ThreadPlanes> planes_;
    std::vector<void*> opened_;  // peer mappings to close
    std::atomic<bool> wedged_{false};
};

}  // namespace switchml

#endif  // SWITCHML_AMD_XGMI_SWITCH_H_
