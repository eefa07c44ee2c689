// loopback_backend.h — the "dummy" backend on MI355X
// (client_lib/src/backends/dummy/dummy_backend.cc, dummy_worker_thread.cc).
//
// Each worker thread owns one PrePostProcessor (and its HIP stream) and runs
// its FIFO slice of every job: pre-process, the loopback "switch" (every
// payload word x num_workers, exponents unchanged: dummy_backend.cc:72-84),
// post-process.  Where the reference moves one 1 KiB packet per call through a
// host ring, this backend moves the whole slice through HBM planes
// (backend.hip.mode = bulk | fused), or — for API parity — runs the
// reference's per-packet call sequence over a device ring (mode = packet).
// Device tensors are used in place, pinned host tensors through their device
// mapping (zero-copy over PCIe); pageable host tensors are staged through
// device buffers (H2D / D2H on the worker's stream).
#ifndef SWITCHML_AMD_LOOPBACK_BACKEND_H_
#define SWITCHML_AMD_LOOPBACK_BACKEND_H_

#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "config.h"
#include "job.h"

namespace switchml {

class Context;
class PrePostProcessor;
class XgmiSwitch;

class LoopbackBackend {
  public:
    LoopbackBackend(Context& context, Config& config);
    ~LoopbackBackend();
    void SetupWorker();    // (xgmi: join the session) start num_worker_threads worker threads
    void CleanupWorker();  // join them (xgmi: leave the session)

  private:
    void WorkerMain(WorkerTid tid);
    // backend.hip.batch_jobs > 0, mode = fused, loopback switch, no simulated
    // wire, HIP pre/post-processor: one thread, batched launches (BatchMain).
    bool BatchEligible() const;
    void BatchMain();

    Context& context_;
    Config& config_;
    std::vector<std::thread> threads_;
    std::mutex wire_mutex_;              // simulated wire time, cut short by Stop()
    std::condition_variable wire_cv_;
    std::unique_ptr<XgmiSwitch> xgmi_;   // general.backend = "xgmi": the in-node switch
};

// True if p is HIP device (or managed) memory; false for host memory.
bool IsDevicePointer(const void* p);
// Address a kernel can use for p: p for device / managed memory, the device
// mapping of pinned host memory, nullptr for pageable host memory.
void* DeviceAddress(void* p);

}  // namespace switchml

#endif  // SWITCHML_AMD_LOOPBACK_BACKEND_H_
