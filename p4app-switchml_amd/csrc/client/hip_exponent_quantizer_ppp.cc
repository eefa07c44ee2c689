// hip_exponent_quantizer_ppp.cc — see hip_exponent_quantizer_ppp.h.
#include "hip_exponent_quantizer_ppp.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <string>

#include "switchml_hip.h"

namespace switchml {

static void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw SwitchMLFatal(std::string(what) + ": " + hipGetErrorString(e));
}

HipExponentQuantizerPPP::HipExponentQuantizerPPP(Config& config, WorkerTid worker_tid, Numel ltu_size,
                                                 Numel batch_num_ltus, bool per_ltu_calls)
    : PrePostProcessor(config, worker_tid, ltu_size, batch_num_ltus), per_ltu_calls_(per_ltu_calls),
      round_flags_(config.backend_.hip.vcl ? SML_FLAG_ROUND_RNE : 0u) {
    ltu_numel_ = ltu_size / 4;
    if (ltu_size % 4 || !(ltu_numel_ == 64 || ltu_numel_ == 128 || ltu_numel_ == 256 || ltu_numel_ == 512 ||
                          ltu_numel_ == 1024))
        throw SwitchMLFatal("hip_exponent_quantizer supports packet_numel 64, 128, 256, 512, 1024; got " +
                            std::to_string(ltu_numel_));
    hip_ok(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
}

HipExponentQuantizerPPP::~HipExponentQuantizerPPP() {
    job_slice_ = nullptr;
    if (abandoned_) return;   // Abandon(): nothing here may wait on the stream's unfinished work
    if (server_) (void)sml_burst_server_destroy(server_);   // no throwing from a destructor
    if (d_recv_exps_) (void)hipFreeAsync(d_recv_exps_, stream_);   // stream-ordered allocation
    if (d_stage_) (void)hipFree(d_stage_);
    if (d_stage_exp_) (void)hipFree(d_stage_exp_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

// The per-LTU trap: a reference worker that keeps
// `prepostprocessor = cpu_exponent_quantizer` and calls PreprocessSingle once
// per 1 KiB packet (DpdkWorkerThread via BuildPacket,
// dpdk_worker_thread_utils.inc:134; RdmaWorkerThread::PostSendWr) would run a
// launch, pointer queries and a host sync per packet — ~14-24 us against the
// CPU loop's ~0.1 us — with no warning.  Under that name the per-LTU calls
// therefore refuse, naming the way out.
void HipExponentQuantizerPPP::refuse_per_ltu(const char* call) const {
    throw SwitchMLFatal(std::string(call) +
                        ": prepostprocessor 'cpu_exponent_quantizer' runs on the MI355X and is driven by its bulk "
                        "hooks (PreprocessBulk / PostprocessBulk) or burst hooks (PreprocessBurst / PostprocessBurst "
                        "/ PostprocessReuseBurst: one launch per rx/tx burst); one call per packet would cost a "
                        "kernel launch and a host sync per 1 KiB packet. Call the burst hooks, or set "
                        "prepostprocessor = hip_exponent_quantizer to accept per-packet launches.");
}

void HipExponentQuantizerPPP::check(int status, const char* what) const {
    if (status != SML_OK)
        throw SwitchMLFatal(std::string(what) + " failed: " + sml_status_string((sml_status_t)status) + " " +
                            sml_last_error());
}

uint64_t HipExponentQuantizerPPP::SetupJobSlice(JobSlice* job_slice) {
    // ppp.cc:54-62
    job_slice_ = job_slice;
    pool_probe_ = nullptr;
    xpool_probe_ = nullptr;
    dev_of_.clear();
    const uint64_t bytes = job_slice->slice.numel * DataTypeSize(job_slice->slice.data_type);
    total_main_num_ltus_ = (bytes + ltu_size_ - 1) / ltu_size_;
    batch_num_ltus_ = std::min<uint64_t>(total_main_num_ltus_, batch_max_num_ltus_);
    return total_main_num_ltus_;
}

bool HipExponentQuantizerPPP::NeedsExtraBatch() { return job_slice_->slice.data_type == FLOAT32; }

void HipExponentQuantizerPPP::CleanupJobSlice() {
    job_slice_ = nullptr;
    server_synced_ = false;
    // a resident server would hold up every device-wide synchronisation:
    // it runs for one slice's packet loop only (its memory and stream stay)
    if (server_ && sml_burst_server_stop(server_) != SML_OK)
        throw SwitchMLFatal(std::string("sml_burst_server_stop: ") + sml_last_error());
}

void HipExponentQuantizerPPP::ensure_single_buffers() {
    if (!d_stage_) {
        hip_ok(hipMalloc(&d_stage_, ltu_size_), "hipMalloc");
        hip_ok(hipMalloc(&d_stage_exp_, 16), "hipMalloc");
    }
    if (d_recv_exps_cap_ < total_main_num_ltus_) {
        // stream-ordered: no device-wide sync on a worker thread (see
        // loopback_backend.cc DeviceBuffer)
        if (d_recv_exps_) hip_ok(hipFreeAsync(d_recv_exps_, stream_), "hipFreeAsync");
        d_recv_exps_ = nullptr;
        d_recv_exps_cap_ = std::max<uint64_t>(total_main_num_ltus_, 1);
        hip_ok(hipMallocAsync(reinterpret_cast<void**>(&d_recv_exps_), d_recv_exps_cap_, stream_), "hipMallocAsync");
    }
}

namespace {

// Where a packet buffer lives, and the address a kernel can use for it:
// device memory and pinned (page-locked, device-mapped) host memory are
// written / read by the kernels directly; pageable host memory is staged.
struct PacketMem {
    void* dev = nullptr;   // kernel-usable address, null for pageable memory
    bool host = true;      // the CPU may touch it right after the call returns
};

PacketMem packet_mem(void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return {};
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return {p, false};
    if (a.type == hipMemoryTypeHost && a.devicePointer) return {a.devicePointer, true};
    return {};
}

}  // namespace

// PreprocessSingle — ppp.cc:69-192.  One kernel per half (quantize of block
// ltu_id - b, exponent of block ltu_id), writing the packet buffer directly
// when the device can address it.  The packet is complete on return, as the
// reference's is, because the caller hands it to the NIC next; only a caller
// that opted into stream order (SetStreamOrdered) with a device-memory packet
// skips the host sync.
void HipExponentQuantizerPPP::PreprocessSingle(uint64_t ltu_id, void* entries_ptr, void* extra_info) {
    if (!per_ltu_calls_) refuse_per_ltu("PreprocessSingle");
    preprocess_single(ltu_id, entries_ptr, extra_info);
}

void HipExponentQuantizerPPP::PostprocessSingle(uint64_t ltu_id, void* entries_ptr, void* extra_info) {
    if (!per_ltu_calls_) refuse_per_ltu("PostprocessSingle");
    postprocess_single(ltu_id, entries_ptr, extra_info);
}

void HipExponentQuantizerPPP::preprocess_single(uint64_t ltu_id, void* entries_ptr, void* extra_info) {
    const Tensor& s = job_slice_->slice;
    const uint32_t P = (uint32_t)ltu_numel_;
    ensure_single_buffers();
    bool sync = false;
    if (s.data_type == FLOAT32) {
        if (ltu_id >= batch_num_ltus_) {
            const uint64_t k = ltu_id - batch_num_ltus_;
            const uint64_t off = k * P, n = std::min<uint64_t>(P, s.numel - off);
            const PacketMem m = packet_mem(entries_ptr);
            sync |= m.host;
            // the kernel writes all P words of the block; the reference writes
            // only the n real ones (ppp.cc:102-109), so a partial block is staged
            int32_t* dst = (m.dev && n == P) ? static_cast<int32_t*>(m.dev) : d_stage_;
            check(sml_quantize_pack(static_cast<const float*>(s.in_ptr) + off, n, P, config_.general_.num_workers,
                                    d_recv_exps_ + k, dst, nullptr, round_flags_, stream_),
                  "sml_quantize_pack");
            if (dst == d_stage_)
                hip_ok(hipMemcpyAsync(entries_ptr, d_stage_, n * 4, hipMemcpyDefault, stream_), "hipMemcpyAsync");
            ltu_id = k + batch_num_ltus_;
        }
        if (ltu_id < total_main_num_ltus_) {
            const uint64_t off = ltu_id * P, n = std::min<uint64_t>(P, s.numel - off);
            const PacketMem m = packet_mem(extra_info);
            sync |= m.host;
            // one byte: the int8 exponent in byte 0 of the extra-info slot (byte 1 untouched)
            int8_t* dst = m.dev ? static_cast<int8_t*>(m.dev) : d_stage_exp_;
            check(sml_exponents(static_cast<const float*>(s.in_ptr) + off, n, P, dst, stream_), "sml_exponents");
            if (dst == d_stage_exp_)
                hip_ok(hipMemcpyAsync(extra_info, d_stage_exp_, 1, hipMemcpyDefault, stream_), "hipMemcpyAsync");
        }
    } else if (s.data_type == INT32) {
        const uint64_t off = ltu_id * P, n = std::min<uint64_t>(P, s.numel - off);
        const PacketMem m = packet_mem(entries_ptr);
        sync |= m.host;
        int32_t* dst = m.dev ? static_cast<int32_t*>(m.dev) : d_stage_;
        check(sml_bswap_i32(static_cast<const int32_t*>(s.in_ptr) + off, dst, n, stream_), "sml_bswap_i32");
        if (dst == d_stage_)
            hip_ok(hipMemcpyAsync(entries_ptr, d_stage_, n * 4, hipMemcpyDefault, stream_), "hipMemcpyAsync");
    } else {
        throw SwitchMLFatal("unsupported data type");
    }
    if (sync || !stream_ordered_) hip_ok(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

// PostprocessSingle — ppp.cc:194-299.  The dequantize kernel reads the packet
// buffer in place when the device can address it (packet buffers hold P
// words, ltu_size bytes); the caller may reuse a host-memory packet buffer
// as soon as this returns, so those calls synchronise.
void HipExponentQuantizerPPP::postprocess_single(uint64_t ltu_id, void* entries_ptr, void* extra_info) {
    const Tensor& s = job_slice_->slice;
    const uint32_t P = (uint32_t)ltu_numel_;
    ensure_single_buffers();
    bool sync = false;
    if (s.data_type == FLOAT32) {
        if (ltu_id >= batch_num_ltus_) {
            const uint64_t k = ltu_id - batch_num_ltus_;
            const uint64_t off = k * P, n = std::min<uint64_t>(P, s.numel - off);
            const PacketMem m = packet_mem(entries_ptr);
            sync |= m.host;
            const int32_t* src = static_cast<const int32_t*>(m.dev);
            if (!src) {
                hip_ok(hipMemcpyAsync(d_stage_, entries_ptr, n * 4, hipMemcpyDefault, stream_), "hipMemcpyAsync");
                src = d_stage_;
            }
            check(sml_dequantize(src, d_recv_exps_ + k, n, P, config_.general_.num_workers,
                                 static_cast<float*>(s.out_ptr) + off, 0, stream_),
                  "sml_dequantize");
            ltu_id = k + batch_num_ltus_;
        }
        if (ltu_id < total_main_num_ltus_) {
            // ppp.cc:254-260 stores the scale of the received exponent; the
            // kernels derive the same scale from the stored exponent.
            sync |= packet_mem(extra_info).host;
            hip_ok(hipMemcpyAsync(d_recv_exps_ + ltu_id, extra_info, 1, hipMemcpyDefault, stream_),
                   "hipMemcpyAsync");
        }
    } else if (s.data_type == INT32) {
        const uint64_t off = ltu_id * P, n = std::min<uint64_t>(P, s.numel - off);
        const PacketMem m = packet_mem(entries_ptr);
        sync |= m.host;
        const int32_t* src = static_cast<const int32_t*>(m.dev);
        if (!src) {
            hip_ok(hipMemcpyAsync(d_stage_, entries_ptr, n * 4, hipMemcpyDefault, stream_), "hipMemcpyAsync");
            src = d_stage_;
        }
        check(sml_bswap_i32(src, static_cast<int32_t*>(s.out_ptr) + off, n, stream_), "sml_bswap_i32");
    } else {
        throw SwitchMLFatal("unsupported data type");
    }
    if (sync || !stream_ordered_) hip_ok(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

// A burst of per-LTU calls as one launch per SML_MAX_BURST packets.  The
// buffers of a burst come from one pool (a ring, a NIC's mbuf pool), so one
// pointer query per burst decides where they live: HBM or pinned host memory
// go to the kernel in place (pinned host memory at its device address — the
// same offset applies to every buffer of the pool); pageable memory takes the
// per-packet path, which stages.
void HipExponentQuantizerPPP::burst(BurstKind kind, uint32_t n, const uint64_t* ltu_ids, void* const* entries,
                                   void* const* extras) {
    if (n == 0) return;
    const Tensor& s = job_slice_->slice;
    const bool flt = s.data_type == FLOAT32;
    const uint64_t total = total_main_num_ltus_ + (flt ? batch_num_ltus_ : 0);
    ensure_single_buffers();
    // one pool per slice: the query is cached for the slice (SetupJobSlice resets it)
    if (entries[0] != pool_probe_) {
        pool_probe_ = entries[0];
        const PacketMem pm = packet_mem(entries[0]);
        pool_dev_ = pm.dev;
        pool_host_ = pm.host;
    }
    const PacketMem m{pool_dev_, pool_host_};
    // the extra-info slots may be another allocation (a separate ring, a
    // second registration): queried on their own
    PacketMem xm{};
    if (extras && extras[0]) {
        if (extras[0] != xpool_probe_) {
            xpool_probe_ = extras[0];
            const PacketMem pm = packet_mem(extras[0]);
            xpool_dev_ = pm.dev;
            xpool_host_ = pm.host;
        }
        xm = {xpool_dev_, xpool_host_};
    }
    if (!m.dev || (extras && extras[0] && !xm.dev)) {
        if (kind == BurstKind::kProcessExchange)
            throw SwitchMLFatal("ProcessPostprocessReuseBurst: packet buffers must be device-addressable");
        for (uint32_t i = 0; i < n; i++) {
            void* x = extras ? extras[i] : nullptr;
            if (kind != BurstKind::kPre) postprocess_single(ltu_ids[i], entries[i], x);
            if (kind == BurstKind::kPre) preprocess_single(ltu_ids[i], entries[i], x);
            else if (kind == BurstKind::kExchange && ltu_ids[i] + batch_num_ltus_ < total)
                preprocess_single(ltu_ids[i] + batch_num_ltus_, entries[i], x);
        }
        return;
    }
    // Host address -> device address: the probe's offset applies to the
    // buffers of its own registration only.  When host and device addresses
    // coincide (HBM, hipHostMalloc) every buffer maps to itself; otherwise (a
    // hipHostRegister'd NIC pool) each buffer is translated by its own query,
    // so buffers of other registrations are never shifted by a wrong offset.
    const intptr_t delta = static_cast<char*>(m.dev) - static_cast<char*>(entries[0]);
    const intptr_t xdelta = xm.dev ? static_cast<char*>(xm.dev) - static_cast<char*>(extras[0]) : 0;
    const bool per_buffer = delta != 0 || xdelta != 0;
    auto dev_addr = [&](void* p) -> void* {
        if (!p || !per_buffer) return p;
        auto it = dev_of_.find(p);   // a NIC pool's buffers recur burst after burst: one query per slice
        if (it != dev_of_.end()) return it->second;
        void* a = packet_mem(p).dev;
        if (!a) throw SwitchMLFatal("burst: a packet buffer of the burst is not device-addressable");
        dev_of_.emplace(p, a);
        return a;
    };
    const bool exchange = kind == BurstKind::kExchange || kind == BurstKind::kProcessExchange;
    sml_packet_burst b{};
    b.in = static_cast<const float*>(s.in_ptr);
    b.out = static_cast<float*>(s.out_ptr);
    b.numel = s.numel;
    b.packet_numel = (uint32_t)ltu_numel_;
    b.num_workers = config_.general_.num_workers;
    b.data_type = flt ? SML_FLOAT32 : SML_INT32;
    // the exchange needs the window for INT32 too (the next packet is q + b)
    b.batch_num_ltus = flt || exchange ? batch_num_ltus_ : 0;
    b.recv_exps = d_recv_exps_;
    b.flags = (kind == BurstKind::kProcessExchange ? SML_FLAG_PROCESS_PACKET : 0u) | round_flags_;
    const char* what = kind == BurstKind::kPre ? "sml_preprocess_burst"
                       : kind == BurstKind::kPost ? "sml_postprocess_burst" : "sml_exchange_burst";
    const bool serve = m.host && config_.backend_.hip.burst_server;
    if (serve && !server_) {
        check(sml_burst_server_create((uint32_t)ltu_numel_, round_flags_, 100, &server_), "sml_burst_server_create");
    }
    if (serve && !server_synced_) {   // the server has its own stream: the slice's staged input must be there
        hip_ok(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        server_synced_ = true;
    }
    const uint32_t op = kind == BurstKind::kPre ? SML_BURST_PRE
                        : kind == BurstKind::kPost ? SML_BURST_POST : SML_BURST_EXCHANGE;
    for (uint32_t i0 = 0; i0 < n; i0 += SML_MAX_BURST) {
        b.count = std::min<uint32_t>(SML_MAX_BURST, n - i0);
        for (uint32_t i = 0; i < b.count; i++) {
            b.pkt_ids[i] = ltu_ids[i0 + i];
            b.entries[i] = dev_addr(entries[i0 + i]);
            b.extras[i] = extras ? dev_addr(extras[i0 + i]) : nullptr;
        }
        if (serve) {   // returns with the burst complete
            check(sml_burst_server_submit(server_, op, &b), "sml_burst_server_submit");
            continue;
        }
        check(kind == BurstKind::kPre ? sml_preprocess_burst(&b, stream_)
              : kind == BurstKind::kPost ? sml_postprocess_burst(&b, stream_) : sml_exchange_burst(&b, stream_),
              what);
    }
    if (serve) return;
    if (m.host || !stream_ordered_) hip_ok(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

void HipExponentQuantizerPPP::PreprocessBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries,
                                              void* const* extras) {
    burst(BurstKind::kPre, n, ltu_ids, entries, extras);
}

void HipExponentQuantizerPPP::PostprocessBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries,
                                               void* const* extras) {
    burst(BurstKind::kPost, n, ltu_ids, entries, extras);
}

void HipExponentQuantizerPPP::PostprocessReuseBurst(uint32_t n, const uint64_t* ltu_ids, void* const* entries,
                                                    void* const* extras, uint64_t batch, uint64_t total_ltus) {
    const bool flt = job_slice_->slice.data_type == FLOAT32;
    if (batch != batch_num_ltus_ || total_ltus != total_main_num_ltus_ + (flt ? batch_num_ltus_ : 0))
        throw SwitchMLFatal("PostprocessReuseBurst: batch / total_ltus differ from the slice's b / B (+ b)");
    burst(BurstKind::kExchange, n, ltu_ids, entries, extras);
}

void HipExponentQuantizerPPP::ProcessPostprocessReuseBurst(uint32_t n, const uint64_t* ltu_ids,
                                                           void* const* entries, void* const* extras) {
    burst(BurstKind::kProcessExchange, n, ltu_ids, entries, extras);
}

void HipExponentQuantizerPPP::ExponentsBulk(void* exps_plane) {
    const Tensor& s = job_slice_->slice;
    if (s.data_type != FLOAT32) return;
    check(sml_exponents(static_cast<const float*>(s.in_ptr), s.numel, (uint32_t)ltu_numel_,
                        static_cast<int8_t*>(exps_plane), stream_),
          "sml_exponents");
}

void HipExponentQuantizerPPP::PreprocessBulk(void* payload_plane, void* exps_plane, const void* global_exps,
                                             bool payload_le) {
    const Tensor& s = job_slice_->slice;
    if (s.data_type == FLOAT32) {
        check(sml_quantize_pack(static_cast<const float*>(s.in_ptr), s.numel, (uint32_t)ltu_numel_,
                                config_.general_.num_workers, static_cast<const int8_t*>(global_exps),
                                static_cast<int32_t*>(payload_plane),
                                global_exps ? nullptr : static_cast<int8_t*>(exps_plane),
                                (payload_le ? SML_FLAG_PAYLOAD_LE : 0u) | round_flags_, stream_),
              "sml_quantize_pack");
    } else {
        if (payload_le)
            hip_ok(hipMemcpyAsync(payload_plane, s.in_ptr, s.numel * 4, hipMemcpyDeviceToDevice, stream_),
                   "hipMemcpyAsync");
        else
            check(sml_bswap_i32(static_cast<const int32_t*>(s.in_ptr), static_cast<int32_t*>(payload_plane),
                                s.numel, stream_),
                  "sml_bswap_i32");
    }
}

void HipExponentQuantizerPPP::PostprocessBulk(const void* payload_plane, const void* global_exps, bool payload_le) {
    const Tensor& s = job_slice_->slice;
    if (s.data_type == FLOAT32) {
        check(sml_dequantize(static_cast<const int32_t*>(payload_plane), static_cast<const int8_t*>(global_exps),
                             s.numel, (uint32_t)ltu_numel_, config_.general_.num_workers,
                             static_cast<float*>(s.out_ptr), payload_le ? SML_FLAG_PAYLOAD_LE : 0u, stream_),
              "sml_dequantize");
    } else {
        if (payload_le)
            hip_ok(hipMemcpyAsync(s.out_ptr, payload_plane, s.numel * 4, hipMemcpyDeviceToDevice, stream_),
                   "hipMemcpyAsync");
        else
            check(sml_bswap_i32(static_cast<const int32_t*>(payload_plane), static_cast<int32_t*>(s.out_ptr),
                                s.numel, stream_),
                  "sml_bswap_i32");
    }
}

int PrePostProcessor::PerLtuCalls(const std::string& name) {
    if (name == "hip_exponent_quantizer" || name == "bypass") return 1;
    if (name == "cpu_exponent_quantizer") return 0;   // bulk / burst hooks only (refuse_per_ltu)
    return -1;
}

std::shared_ptr<PrePostProcessor> PrePostProcessor::CreateInstance(Config& config, WorkerTid worker_tid,
                                                                   Numel ltu_size, Numel batch_num_ltus) {
    const std::string& name = config.general_.prepostprocessor;
    const int per_ltu = PerLtuCalls(name);
    if (per_ltu < 0) throw SwitchMLFatal("'" + name + "' is not a valid prepostprocessor.");
    if (name == "bypass") return std::make_shared<BypassPPP>(config, worker_tid, ltu_size, batch_num_ltus);
    return std::make_shared<HipExponentQuantizerPPP>(config, worker_tid, ltu_size, batch_num_ltus, per_ltu == 1);
}

}  // namespace switchml
