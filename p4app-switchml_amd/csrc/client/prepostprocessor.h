// prepostprocessor.h — the PrePostProcessor (PPP) interface
// (client_lib/src/prepostprocessor.h:44-147) with the bulk hooks the
// reference reserved but never defined (prepostprocessor.h:112-116).
//
// Per-LTU calls (PreprocessSingle / PostprocessSingle) keep the reference's
// exact contract so packet-driven backends can call them, one packet or one
// burst of packets per call; the bulk calls are how a GPU PPP is driven best:
// one call per job slice, planes in HBM.
#ifndef SWITCHML_AMD_PREPOSTPROCESSOR_H_
#define SWITCHML_AMD_PREPOSTPROCESSOR_H_

#include <memory>
#include <string>

#include "common.h"
#include "config.h"
#include "job.h"

namespace switchml {

class PrePostProcessor {
  public:
    // Factory keyed by config.general_.prepostprocessor (prepostprocessor.cc:32-41):
    //   "hip_exponent_quantizer"  -> HipExponentQuantizerPPP (MI355X kernels)
    //   "cpu_exponent_quantizer"  -> HipExponentQuantizerPPP as well: the drop-in
    //                                name of the reference's quantizer, same bytes,
    //                                driven by bulk / burst hooks only — its
    //                                PreprocessSingle / PostprocessSingle throw
    //                                (a per-packet caller would pay a launch and
    //                                a host sync per packet)
    //   "bypass"                  -> BypassPPP
    // Anything else throws SwitchMLFatal (the reference: LOG(FATAL)).
    static std::shared_ptr<PrePostProcessor> CreateInstance(Config& config, WorkerTid worker_tid,
                                                            Numel ltu_size, Numel batch_num_ltus);
    // Whether the PPP a factory key names takes per-LTU calls: 1 yes, 0 no
    // (bulk / burst hooks only), -1 not a valid prepostprocessor.
    static int PerLtuCalls(const std::string& name);
    virtual ~PrePostProcessor() = default;
    PrePostProcessor(const PrePostProcessor&) = delete;
    PrePostProcessor& operator=(const PrePostProcessor&) = delete;

    // Returns the number of LTUs (packets) of the slice, excluding the extra batch.
    virtual uint64_t SetupJobSlice(JobSlice* job_slice) = 0;
    virtual bool NeedsExtraBatch() = 0;
    virtual void PreprocessSingle(uint64_t ltu_id, void* entries_ptr, void* extra_info = nullptr) = 0;
    virtual void PostprocessSingle(uint64_t ltu_id, void* entries_ptr, void* extra_info = nullptr) = 0;
    virtual void CleanupJobSlice() = 0;

    // ---- bulk hooks (one call per job slice; planes are DEVICE memory) ----
    // The planes: exps[B] (int8) and payload[B * ltu_numel] (int32, big-endian
    // wire words unless payload_le), see include/switchml_hip.h.
    //
    // Exponent plane only (the values the first batch of packets would carry).
    virtual void ExponentsBulk(void* exps_plane) { (void)exps_plane; }
    // Quantize + pack every LTU of the slice.  global_exps == nullptr: use the
    // slice's own exponents (loopback: the switch returns them unchanged) and
    // write them to exps_plane; otherwise quantize with the aggregated ones.
    virtual void PreprocessBulk(void* payload_plane, void* exps_plane, const void* global_exps,
                                bool payload_le = false) = 0;
    // Dequantize the aggregated payload with the aggregated exponents into
    // the slice's out_ptr.
    virtual void PostprocessBulk(const void* payload_plane, const void* global_exps,
                                 bool payload_le = false) = 0;

    // ---- burst hooks: the per-LTU calls for n packets at once ----
    // Same contract as n calls of PreprocessSingle(ltu_ids[i], entries[i],
    // extras[i]) (PostprocessSingle) in that order — the packets of one DPDK
    // rx burst and the tx burst it refills (dpdk_worker_thread.cc:276-345),
    // or one RDMA completion batch.  This default is that loop; the HIP PPP
    // runs a burst as one launch.
    virtual void PreprocessBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries, void* const* extras) {
        for (uint32_t i = 0; i < n; i++) PreprocessSingle(ltu_ids[i], entries[i], extras ? extras[i] : nullptr);
    }
    virtual void PostprocessBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries, void* const* extras) {
        for (uint32_t i = 0; i < n; i++) PostprocessSingle(ltu_ids[i], entries[i], extras ? extras[i] : nullptr);
    }
    // The receive loop's two calls on one buffer: for every received packet
    // q = ltu_ids[i], PostprocessSingle(q) and then, when q + batch <
    // total_ltus, PreprocessSingle(q + batch) into the same entries[i] /
    // extras[i] — DpdkWorkerThread's PostprocessSingle + ReusePacket
    // (dpdk_worker_thread.cc:300-345, dpdk_worker_thread_utils.inc:134,177) and
    // DummyWorkerThread's loop trip (dummy_worker_thread.cc:106-163).
    // total_ltus = B, plus b when NeedsExtraBatch().  This default is that
    // loop; the HIP PPP runs it as one launch per burst.
    virtual void PostprocessReuseBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries,
                                       void* const* extras, uint64_t batch, uint64_t total_ltus) {
        for (uint32_t i = 0; i < n; i++) {
            void* x = extras ? extras[i] : nullptr;
            PostprocessSingle(ltu_ids[i], entries[i], x);
            if (ltu_ids[i] + batch < total_ltus) PreprocessSingle(ltu_ids[i] + batch, entries[i], x);
        }
    }

    Numel ltu_size() const { return ltu_size_; }

  protected:
    PrePostProcessor(Config& config, WorkerTid worker_tid, Numel ltu_size, Numel batch_num_ltus)
        : config_(config), worker_tid_(worker_tid), ltu_size_(ltu_size), batch_max_num_ltus_(batch_num_ltus) {}

    Config& config_;
    WorkerTid worker_tid_;
    Numel ltu_size_;            // bytes per LTU
    Numel batch_max_num_ltus_;  // max LTUs per batch
};

// bypass_ppp.h:40-105: counts LTUs, moves no data (packets carry garbage).
class BypassPPP : public PrePostProcessor {
  public:
    BypassPPP(Config& c, WorkerTid t, Numel ltu, Numel batch) : PrePostProcessor(c, t, ltu, batch) {}
    uint64_t SetupJobSlice(JobSlice* s) override {
        const uint64_t bytes = s->slice.numel * DataTypeSize(s->slice.data_type);
        return (bytes + ltu_size_ - 1) / ltu_size_;
    }
    bool NeedsExtraBatch() override { return false; }
    void PreprocessSingle(uint64_t, void*, void*) override {}
    void PostprocessSingle(uint64_t, void*, void*) override {}
    void CleanupJobSlice() override {}
    void PreprocessBulk(void*, void*, const void*, bool) override {}
    void PostprocessBulk(const void*, const void*, bool) override {}
};

}  // namespace switchml

#endif  // SWITCHML_AMD_PREPOSTPROCESSOR_H_
