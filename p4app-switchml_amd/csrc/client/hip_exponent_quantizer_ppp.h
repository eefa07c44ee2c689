// hip_exponent_quantizer_ppp.h — SwitchML's exponent quantizer PPP on MI355X.
//
// Same contract as CpuExponentQuantizerPPP
// (client_lib/src/prepostprocessors/cpu_exponent_quantizer_ppp.{h,cc}), with
// the arithmetic done by the gfx950 kernels behind include/switchml_hip.h:
//   * per-LTU calls keep the reference's packet semantics exactly (packet p
//     carries the exponent of block p, p < B, and the payload of block p - b,
//     p >= b; the scale of block k comes from the exponent received with
//     packet k) — one small kernel launch per call, or per BURST of packets
//     (a DPDK rx / tx burst) for packet-driven callers;
//   * bulk calls process the whole slice in one launch (the fast path).
// The job slice's in_ptr / out_ptr must be DEVICE memory (the loopback
// backend stages host tensors); entries / extra-info pointers of the
// per-LTU calls may be host or device memory.
#ifndef SWITCHML_AMD_HIP_EXPONENT_QUANTIZER_PPP_H_
#define SWITCHML_AMD_HIP_EXPONENT_QUANTIZER_PPP_H_

#include <hip/hip_runtime_api.h>

#include <unordered_map>

#include "prepostprocessor.h"
#include "switchml_hip.h"

namespace switchml {

class HipExponentQuantizerPPP : public PrePostProcessor {
  public:
    // per_ltu_calls = false: PreprocessSingle / PostprocessSingle called from
    // outside (a reference worker's per-packet loop) throw instead of running
    // one launch + host sync per packet; bulk and burst hooks are unaffected.
    HipExponentQuantizerPPP(Config& config, WorkerTid worker_tid, Numel ltu_size, Numel batch_num_ltus,
                            bool per_ltu_calls = true);
    ~HipExponentQuantizerPPP() override;

    uint64_t SetupJobSlice(JobSlice* job_slice) override;
    bool NeedsExtraBatch() override;
    void PreprocessSingle(uint64_t ltu_id, void* entries_ptr, void* extra_info) override;
    void PostprocessSingle(uint64_t ltu_id, void* entries_ptr, void* extra_info) override;
    void CleanupJobSlice() override;

    // One launch per burst of up to SML_MAX_BURST packets (sml_preprocess_burst
    // / sml_postprocess_burst): the packet buffers must be device-addressable
    // (HBM or pinned host memory); pageable ones take the per-packet path.
    void PreprocessBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries, void* const* extras) override;
    void PostprocessBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries, void* const* extras) override;
    // One launch per SML_MAX_BURST received packets (sml_exchange_burst);
    // batch / total_ltus must be this slice's b and B (+ b for FLOAT32).
    void PostprocessReuseBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries, void* const* extras,
                               uint64_t batch, uint64_t total_ltus) override;
    // The same with the dummy backend's ProcessPacket (x num_workers,
    // dummy_backend.cc:72-84) applied to each packet first, in the same launch:
    // the loopback backend's device ring runs a whole ring pass as one launch.
    void ProcessPostprocessReuseBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries,
                                      void* const* extras);

    // A per-LTU / burst call returns with its packet complete, as the
    // reference's does (the caller hands a packet to the NIC next).  A caller
    // whose packets stay in HBM and are consumed on stream() (the loopback
    // backend's device ring) may opt out of the host sync.
    void SetStreamOrdered(bool on) { stream_ordered_ = on; }

    void ExponentsBulk(void* exps_plane) override;
    void PreprocessBulk(void* payload_plane, void* exps_plane, const void* global_exps, bool payload_le) override;
    void PostprocessBulk(const void* payload_plane, const void* global_exps, bool payload_le) override;

    hipStream_t stream() const { return stream_; }
    // Work on stream() did not finish within a bounded wait (the in-node
    // switch's timeout) and may never: the destructor then leaks the stream
    // and the device buffers instead of freeing them (hipFree /
    // hipStreamDestroy would wait on that work).
    void Abandon() { abandoned_ = true; }
    uint64_t total_main_num_ltus() const { return total_main_num_ltus_; }
    uint64_t batch_num_ltus() const { return batch_num_ltus_; }
    Numel ltu_numel() const { return ltu_numel_; }

  private:
    void check(int status, const char* what) const;
    void refuse_per_ltu(const char* call) const;
    void preprocess_single(uint64_t ltu_id, void* entries_ptr, void* extra_info);
    void postprocess_single(uint64_t ltu_id, void* entries_ptr, void* extra_info);
    void ensure_single_buffers();
    enum class BurstKind { kPre, kPost, kExchange, kProcessExchange };
    void burst(BurstKind kind, uint32_t n, const uint64_t* ltu_ids, void* const* entries, void* const* extras);

    JobSlice* job_slice_ = nullptr;
    uint64_t total_main_num_ltus_ = 0;  // B
    uint64_t batch_num_ltus_ = 0;       // b
    Numel ltu_numel_ = 0;               // P (elements per LTU)
    hipStream_t stream_ = nullptr;
    // per-LTU mode state: received (global) exponents of the slice, and
    // device staging for one LTU of entries / one exponent byte
    int8_t* d_recv_exps_ = nullptr;
    uint64_t d_recv_exps_cap_ = 0;
    int32_t* d_stage_ = nullptr;
    int8_t* d_stage_exp_ = nullptr;
    bool stream_ordered_ = false;
    bool abandoned_ = false;
    bool per_ltu_calls_ = true;
    // SML_FLAG_ROUND_RNE when backend.hip.vcl (the reference's VCL=1 build's
    // rounding), else 0: or'ed into every quantizing launch
    uint32_t round_flags_ = 0;
    // where the slice's packet pool lives (burst calls): the first buffer
    // pointer seen, and its packet_mem() answer — for the entries and, as a
    // separate query, the extra-info slots (they may be another allocation)
    void* pool_probe_ = nullptr;
    void* pool_dev_ = nullptr;
    bool pool_host_ = true;
    void* xpool_probe_ = nullptr;
    void* xpool_dev_ = nullptr;
    bool xpool_host_ = true;
    // host -> device address of each packet buffer of the slice, when the
    // pool's addresses differ (a hipHostRegister'd pool): queried per buffer
    std::unordered_map<void*, void*> dev_of_;
    // persistent burst server for host-memory packets (backend.hip.burst_server)
    sml_burst_server* server_ = nullptr;
    bool server_synced_ = false;   // stream_ drained before the slice's first server burst
};

}  // namespace switchml

#endif  // SWITCHML_AMD_HIP_EXPONENT_QUANTIZER_PPP_H_
